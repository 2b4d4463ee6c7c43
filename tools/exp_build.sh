# Experiment builds: libdfk_<tag>.so with one source recompiled under extra -D flags (tools only; selected
# by DFK_LIB=...). Usage: bash tools/exp_build.sh <tag> <source.hip> -DFLAG ...
set -e
tag=$1; src=$2; shift 2
root=$(cd "$(dirname "$0")/.." && pwd)
python -m deepfake_amd.build > /dev/null
b=$root/deepfake_amd/build; o=$b/exp_$tag.o
extra=""
[ "$src" = wattn.hip ] && extra=${WATTN_FLAGS-"-mllvm -amdgpu-mfma-vgpr-form=1 -fno-honor-nans -mno-amdgpu-ieee"}
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -Wno-unused-result $extra "$@" -c $root/deepfake_amd/csrc/$src -o $o
objs=$(ls $b/*.o | grep -v "/exp_" | grep -v "/${src%.hip}.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $root/deepfake_amd/libdfk_$tag.so $objs $o
echo built libdfk_$tag.so
