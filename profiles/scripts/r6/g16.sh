#!/bin/bash
# round 6, call 16: arena tests (plain overflow) + GPT-3 medium's largest step allocations
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g16; mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -X faulthandler -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_arena_gpu.py > $O/tests.txt 2>&1
rc=$?; tail -4 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
PYTHONPATH=$R timeout -k 10 300 python3 -u tools/mem_audit.py gpt3 --trace > $O/gpt_audit.txt 2>&1
rc=$?; grep "step_alloc\|base_site" $O/gpt_audit.txt | head -30; exit $rc
