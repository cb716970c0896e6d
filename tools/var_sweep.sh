# usage: bash tools/var_sweep.sh OUT.log OPS variant...   (variant "base" = in-tree library)
out=$1; ops=$2; shift 2
for v in "$@"; do
  if [ $v = base ]; then unset RGAN_LIB; else export RGAN_LIB=$PWD/tools/variants/librgan_$v.so; fi
  echo "== $v" >> $out
  timeout -k 10 120 python tools/gemm_micro.py 20 $ops >> $out 2>&1 || exit $?
done
