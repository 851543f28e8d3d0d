# Build libacf_apr.so from the CURRENT sources with extra -D flags into
# tools/libacf_apr_<name>.so, for same-box A/Bs of a constant (tools/gpu_ab_large.sh).
# usage: bash tools/build_variant.sh <name> "-DACF_FOO=1 ..."
set -e
cd "$(dirname "$0")/.."
S=adversarial-collaborative-filtering_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -Wall -Wno-unused-result \
  $2 -I include $S/acf_apr.hip $S/acf_ops.hip -o tools/libacf_apr_$1.so
echo tools/libacf_apr_$1.so
