#!/bin/bash
# round 6, call 34: whole GPU tier + smoke + default bench on HEAD
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g34; mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tier.txt 2>&1
rc=$?; tail -3 $O/tier.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
rc=$?; tail -1 $O/smoke.txt | cut -c1-200; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/bench.py > $O/bench.jsonl 2> $O/bench.err
rc=$?; tail -1 $O/bench.jsonl | cut -c1-300; exit $rc
