"""CPU oracle for the DeepFake fused-model hot path — TEST INFRASTRUCTURE ONLY.

A functional, pure-torch fp32 CPU restatement of the reference algorithm
(Polarisjame/DeepFake @ 2024_10_08; wav2vec2 from transformers 5.15.0), each
function citing the reference file:line it restates.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it, and only as the checker / the timed CPU baseline — the product package
``deepfake_amd`` never imports it and fails loudly without its HIP library.

Parity pinning: the restatement is checked against golden vectors produced by
importing the reference modules themselves in the build container
(tests/golden/make_golden.py, fixtures in tests/golden/*.npz).  wav2vec2 is
third-party (transformers, unpinned by the reference): it is
pinned to the container's transformers 5.15.0 through the same fixtures.
"""
