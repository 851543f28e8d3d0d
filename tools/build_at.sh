# Build libacf_apr.so from an older commit's sources into tools/libacf_apr_<rev>.so
# (same-box A/Bs against the current build: tools/large_line.py, ACF_LARGE_LINE_LIB).
# usage: bash tools/build_at.sh <rev>
set -e
cd "$(dirname "$0")/.."
rev=$1
tmp=$(mktemp -d)
mkdir -p $tmp/include $tmp/csrc
git show $rev:include/acf_apr.h > $tmp/include/acf_apr.h
for f in $(git ls-tree --name-only $rev adversarial-collaborative-filtering_amd/csrc/); do
  case $f in *.hip|*.h) git show $rev:$f > $tmp/csrc/$(basename $f);; esac
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -I $tmp/include \
  $tmp/csrc/acf_apr.hip $tmp/csrc/acf_ops.hip -o tools/libacf_apr_$rev.so
rm -rf $tmp
echo tools/libacf_apr_$rev.so
