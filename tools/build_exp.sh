# Experiment libraries (not the product): libnkvmerkle_<tag>.so with extra -D flags.
#   bash tools/build_exp.sh <tag> -DFOO=1 ...
set -e
tag=$1; shift
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -pthread -Wall -Wno-unused-result \
  -I include -I nakevaleng_amd/csrc "$@" nakevaleng_amd/csrc/kernels.hip nakevaleng_amd/csrc/crc.hip \
  nakevaleng_amd/csrc/bloom.hip nakevaleng_amd/csrc/capi.cpp nakevaleng_amd/csrc/host_stage.cpp \
  nakevaleng_amd/csrc/group.cpp -L/opt/rocm/lib -lrccl -lhsa-runtime64 \
  -o tools/libnkvmerkle_$tag.so
