#!/bin/bash
# variants vs the in-tree library on C4 only.  usage: tools/gpu_r4t.sh TAG NAME...
set -u
tag=${1:-r4t}; shift
stop() { case $1 in 124|134|137|139) echo "STOP: rc=$1 at $2"; exit "$1" ;; esac; }
for v in "$@"; do
  timeout -k 10 400 tools/ab_lib.sh "$tag" C4 $v 20; rc=$?; stop $rc ab_C4_$v; [ $rc -eq 0 ] || exit $rc
done
