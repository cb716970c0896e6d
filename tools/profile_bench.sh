#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run (GPU box).  usage: tools/profile_bench.sh OUTDIR [bench args]
set -e
out=$(realpath -m "$1"); shift
root=$(pwd)
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$out" -o run --output-format csv -- python3 "$root/bench.py" "$@" > "$out/bench.log" 2>&1
python3 "$root/profiles/summarize.py" "$out" > "$out/summary.txt"
# provenance: the commit the snapshot was taken from (BUILD_HEAD, written before gpurun) and the command
echo "# head $(cat "$root/BUILD_HEAD" 2>/dev/null || echo unknown); bench.py $*" >> "$out/summary.txt"
