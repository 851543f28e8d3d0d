# k_stream critical-path diagnostics (stamped build)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${OUT_TAG:-stream_diag}
mkdir -p $OUT
NB=200 timeout -k 10 200 python3 tools/diag_stream.py > $OUT/diag.json 2> $OUT/diag.err
cat $OUT/diag.json
