#!/bin/bash
# round 6, call 45: FFConfig.device_arena + refactored arena sizing -- arena tests, the default bench, whole GPU tier
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g45; mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_arena_gpu.py > $O/arena.txt 2>&1
rc=$?; tail -5 $O/arena.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tier.txt 2>&1
rc=$?; tail -2 $O/tier.txt; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/bench.py > $O/bench.jsonl 2> $O/bench.err
rc=$?; tail -1 $O/bench.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print(d['value'], d['ms_per_step'], c['global_batch'], c['memory'].get('device_arena'))"; exit $rc
