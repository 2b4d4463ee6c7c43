set -e
mkdir -p gpurun_out/pe
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_vst.py tests/test_gpu_im2col.py > gpurun_out/pe/tests.log 2>&1
for pc in 1 2 3; do for d in 1 2; do
  DFK_PE_PERCU=$pc DFK_PE_DEPTH=$d timeout -k 10 120 python tools/pe_bench.py >> gpurun_out/pe/sweep.log 2>&1
done; done
cat gpurun_out/pe/sweep.log; tail -3 gpurun_out/pe/tests.log
