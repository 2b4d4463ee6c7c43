set -o pipefail
mkdir -p gpurun_out/bt
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_wattn.py tests/test_gpu_vst.py > gpurun_out/bt/tests.log 2>&1; rc=$?; tail -5 gpurun_out/bt/tests.log; [ $rc = 0 ] || exit $rc
for v in "DFK_WATTN_BWD_OLD=1" "DFK_WATTN_BWD_DET=1" "DFK_WATTN_BWD_DET=0"; do echo "== $v"; env $v timeout -k 10 120 python tools/wattn_bench.py 20 2>&1 | grep -v amdgpu.ids; done
