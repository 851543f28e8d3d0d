# -DACF_DIAG build of the step library for tools/diag_*.py (stamps; diagnostics only)
set -e
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -DACF_DIAG -I include \
  adversarial-collaborative-filtering_amd/csrc/acf_apr.hip adversarial-collaborative-filtering_amd/csrc/acf_ops.hip \
  -o tools/libacf_apr_diag.so
