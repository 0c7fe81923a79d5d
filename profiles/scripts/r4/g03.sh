# round 4, call 3: measured per-op cost tables at the current kernels for the
# four bench configs (simulator calibration, tools/search_report.py); tables
# are written after every op, so a step cut by its limit keeps its rows
set -o pipefail
mkdir -p gpurun_out/prof_tables
M=${1:-bert-large}; W=${2:-8}
timeout -k 10 1000 python -u tools/profile_ops.py --model $M --world $W --out gpurun_out/prof_tables/op_costs_${M}_w${W}_r4.json 2>&1 | tee gpurun_out/prof_tables/$M.log
