# A/B of one environment toggle on the same box:  bash tools/ab_env.sh VAR "bench args" out_name
# Runs bench.py with VAR=0 and VAR=1 twice each (interleaved), lines into gpurun_out/<out_name>.txt
set -o pipefail
VAR=$1; ARGS=$2; OUT=gpurun_out/$3.txt
: > $OUT
for rep in 1 2; do
  for v in 0 1; do
    line=$(env $VAR=$v timeout -k 10 300 python -u bench.py $ARGS 2>gpurun_out/$3.err | tail -1) || exit 1
    echo "$VAR=$v $line" >> $OUT
  done
done
