#!/bin/bash
# GPU-box half of tools/wprobe.py: a kernel-trace pass and one rocprofv3 --pmc pass per counter set, each
# with its own time limit. Summarise with: python3 tools/wprobe_summary.py gpurun_out/wprobe/<tag>
set -o pipefail
tag=${1:-w}
shift || true
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/wprobe/$tag
mkdir -p "$out"
timeout -k 10 240 rocprofv3 --kernel-trace -d "$out/trace" -o run -f csv -- python3 tools/wprobe.py "$@" > "$out/wprobe.json" 2> "$out/trace.err" \
    || { echo "trace pass failed"; tail -20 "$out/trace.err"; exit 1; }
for pass in "fetch FETCH_SIZE" "write WRITE_SIZE" "wreq TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
    set -- $pass
    name=$1; shift
    timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-include-regex ngx_jit_final -d "$out/$name" -o run -f csv -- \
        python3 tools/wprobe.py > "$out/$name.json" 2> "$out/$name.err" || { echo "$name pass failed"; tail -5 "$out/$name.err"; [ $name = wreq ] || exit 1; }
done
python3 tools/wprobe_summary.py "$out"
