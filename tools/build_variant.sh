# Build an A/B variant of libfrei_hip.so with extra compile definitions.
#   bash tools/build_variant.sh OUT.so [-DNAME=VALUE ...]
set -e
OUT=$1; shift
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -fPIC -shared -std=c++17 \
  -Iinclude "$@" frei_amd/csrc/frei_kernels.hip frei_amd/csrc/frei_runtime.hip \
  frei_amd/csrc/frei_binning.hip -o "$OUT" -ldl
