#!/bin/bash
# split-K planner variants vs the in-tree library on C4 and C1
set -u
tag=${1:-r4r}; shift
stop() { case $1 in 124|134|137|139) echo "STOP: rc=$1 at $2"; exit "$1" ;; esac; }
for v in "$@"; do
  for wl in C4 C1; do
    timeout -k 10 400 tools/ab_lib.sh "$tag" $wl $v 20; rc=$?; stop $rc ab_${wl}_$v; [ $rc -eq 0 ] || exit $rc
  done
done
