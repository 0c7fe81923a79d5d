#!/bin/bash
# round 6, call 31: the whole multi-rank bench flow over RCCL at world 1 (calibration, DP reference, AE protocol:
# five models built, captured and replayed in one process with the RCCL watchdog alive)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g31; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
FF_DIST_WORLD1=1 FF_BENCH_REHEARSE_MULTI=1 timeout -k 10 500 python3 $R/bench.py --steps 10 --warmup 3 > $O/bench.jsonl 2> $O/bench.err \
  || { grep -v "^frame" $O/bench.err | tail -20; exit 1; }
tail -1 $O/bench.jsonl | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['config']
print(d['value'], d['ms_per_step'], d['world_size'], d['backend'], c['parallelism'], c.get('graph_segments'), c.get('native_replay'))
for k in ('comm_calibration','dp_samples_per_sec','speedup_over_dp','dp_reference','ae_bert','ae_speedup_over_dp','after_headline'):
    print(k, json.dumps(c.get(k))[:400])"
