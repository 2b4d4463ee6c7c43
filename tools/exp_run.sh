# run a tool against each experiment build: bash tools/exp_run.sh "<cmd>" tag1 tag2 ...  (tag "base" = libdfk.so)
set -o pipefail
cmd=$1; shift
mkdir -p gpurun_out/exp
for t in "$@"; do
  if [ "$t" = base ]; then lib=""; else lib=$PWD/deepfake_amd/libdfk_$t.so; fi
  echo "== $t" | tee -a gpurun_out/exp/log.txt
  DFK_LIB=$lib timeout -k 10 120 $cmd 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/exp/log.txt || exit 1
done
