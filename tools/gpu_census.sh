cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/census
timeout -k 10 300 python3 -u tools/gemm_census.py > gpurun_out/census/census.txt 2>&1 && \
timeout -k 10 300 python3 -u tools/gemm_bench.py --torch > gpurun_out/census/gemm_bench.txt 2>&1
