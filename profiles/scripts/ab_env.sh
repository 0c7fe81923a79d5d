# A/B of one environment toggle on the same box:
#   bash profiles/scripts/ab_env.sh VAR "bench args" out_name [value_a value_b]
# Runs bench.py with VAR=a and VAR=b twice each (interleaved), lines into gpurun_out/<out_name>.txt
set -o pipefail
VAR=$1; ARGS=$2; OUT=gpurun_out/$3.txt
A=${4:-0}; B=${5:-1}
: > $OUT
for rep in 1 2; do
  for v in $A $B; do
    line=$(env $VAR=$v timeout -k 10 300 python -u bench.py $ARGS 2>gpurun_out/$3.err | tail -1) || exit 1
    echo "$VAR=$v $line" >> $OUT
  done
done
