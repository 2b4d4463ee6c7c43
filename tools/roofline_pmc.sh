# PMC passes (one counter group per rocprofv3 run) for bench.py's roofline kernel -> profiles/<tag>_wattn_fwd_pmc.json
set -o pipefail
tag=${1:-r2}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/pmc_roof; mkdir -p $out
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $out/f -o run --output-format csv -- python3 tools/roofline_pmc.py run 5 > $out/f.log 2>&1 || { tail $out/f.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $out/w -o run --output-format csv -- python3 tools/roofline_pmc.py run 5 > $out/w.log 2>&1 || { tail $out/w.log; exit 1; }
python3 tools/roofline_pmc.py parse $(find $out/f -name run_counter_collection.csv) $(find $out/w -name run_counter_collection.csv) $out/${tag}_wattn_fwd_pmc.json
