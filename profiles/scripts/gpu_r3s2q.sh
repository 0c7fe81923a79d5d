# One-clock autotuning (all candidates graph-timed when the fastest is < 50 us): tests, DLRM, BERT / ResNet A/B.
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/gt3_tests.log 2>&1 || exit $?
FF_GEMM_REPORT=1 timeout -k 10 300 python -u bench.py --model dlrm --steps 20 --warmup 5 > gpurun_out/gt3_dlrm.log 2> gpurun_out/gt3_dlrm_report.txt || exit $?
timeout -k 10 300 python -u bench.py --model dlrm --steps 20 --warmup 5 >> gpurun_out/gt3_dlrm.log 2>/dev/null || exit $?
bash tools/ab_env.sh FF_AUTOTUNE_GRAPH "--steps 10 --warmup 3" ab_autotune_graph3_bert || exit $?
bash tools/ab_env.sh FF_AUTOTUNE_GRAPH "--model resnet50 --steps 20 --warmup 5" ab_autotune_graph3_resnet
