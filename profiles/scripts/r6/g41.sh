#!/bin/bash
# round 6, call 41: the default bench (BERT-large, 128 sequences / GPU) and the multi-rank flow over RCCL at world 1
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g41; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/bench.py > $O/default.jsonl 2> $O/default.err || { tail -5 $O/default.err; exit 1; }
tail -1 $O/default.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print(d['value'], d['ms_per_step'], c['global_batch'], c['memory'])"
FF_DIST_WORLD1=1 FF_BENCH_REHEARSE_MULTI=1 timeout -k 10 500 python3 $R/bench.py > $O/rccl1.jsonl 2> $O/rccl1.err || { grep -v "^frame" $O/rccl1.err | tail -10; exit 1; }
tail -1 $O/rccl1.jsonl | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['config']
print(d['value'], d['ms_per_step'], d['world_size'], d['backend'], c['parallelism'], c.get('graph_segments'), c.get('native_replay'))
for k in ('speedup_over_dp','dp_samples_per_sec','dp_reference','ae_bert','ae_speedup_over_dp','after_headline'):
    print(' ', k, json.dumps(c.get(k))[:400])"
