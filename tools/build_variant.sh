# Build an A/B variant of libfrei_hip.so with extra compile definitions.
#   bash tools/build_variant.sh OUT.so [-DNAME=VALUE ...]
# A -D switch that no source under frei_amd/csrc/ names fails the build: a retired switch would
# otherwise compile the default kernels and an A/B would compare identical code.
set -e
OUT=$1; shift
cd "$(dirname "$0")/.."
for d in "$@"; do
  case "$d" in
    -D*) name=${d#-D}; name=${name%%=*}
         grep -rqw -- "$name" frei_amd/csrc/ || { echo "build_variant: $name is not referenced in frei_amd/csrc" >&2; exit 2; } ;;
  esac
done
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -fPIC -shared -std=c++17 \
  -Iinclude "$@" frei_amd/csrc/frei_kernels.hip frei_amd/csrc/frei_runtime.hip \
  frei_amd/csrc/frei_binning.hip -o "$OUT" -ldl
