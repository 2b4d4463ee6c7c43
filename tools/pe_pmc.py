"""PMC bytes of the fused PatchEmbed3D forward launches of a bench.py run (rocprofv3 --pmc FETCH_SIZE, then
WRITE_SIZE + TCC_EA0_WRREQ_sum): the in-step launches (inside the replayed training step) against the roofline
loop's cold launches (the last ones), per launch, with the gfx950 correction of FETCH_SIZE (x2 for 16-B-per-lane
reads, MI355X_MICROARCH.md HBM / rocprofv3 section).  usage: pe_pmc.py fetch.csv write.csv"""
import csv
import statistics
import sys


def rows(path, counter):
    out = []
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter and "pe_fwd_kernel" in r["Kernel_Name"]:
            out.append((int(r.get("Dispatch_Id", 0) or 0), float(r["Counter_Value"])))
    return [v for _, v in sorted(out)]


def main(fcsv, wcsv):
    f, w, q = rows(fcsv, "FETCH_SIZE"), rows(wcsv, "WRITE_SIZE"), rows(wcsv, "TCC_EA0_WRREQ_sum")
    # bench.py order: warm-up + timed steps (one launch each; the captured step replays its launch), then the
    # roofline loop (1 + roofline-iters launches): the last 7 are the cold isolated loop
    n_iso = 7
    for name, v in (("FETCH_SIZE KiB", f), ("WRITE_SIZE KiB", w), ("TCC_EA0_WRREQ", q)):
        step, iso = v[:-n_iso], v[-n_iso:]
        print(f"{name:16s} in-step n={len(step)} median {statistics.median(step) if step else float('nan'):.1f}   "
              f"isolated n={len(iso)} median {statistics.median(iso):.1f}")
    print("FETCH_SIZE is reported x2 on gfx950 for 16-B-per-lane reads; bytes = KiB * 1024")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
