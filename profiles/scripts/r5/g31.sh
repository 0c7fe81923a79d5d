# round 5, call 31: 2-rank rehearsal on one GPU (gloo, searched hybrid strategy, segmented hipGraph
# steps) with the native replay, then with the Python walk
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5g31; mkdir -p $O
timeout -k 10 600 bash profiles/scripts/rehearse_multi.sh 2 bert-large > $O/native.jsonl 2> $O/native.err || { tail -30 $O/native.err; exit 1; }
grep -o '"value": [0-9.]*\|"graph_segments": [^]]*]\|"native_replay": [a-z]*\|"final_loss": [0-9.]*' $O/native.jsonl | tr '\n' ' '; echo
FF_NATIVE_REPLAY=0 timeout -k 10 600 bash profiles/scripts/rehearse_multi.sh 2 bert-large > $O/python.jsonl 2> $O/python.err || { tail -30 $O/python.err; exit 1; }
grep -o '"value": [0-9.]*\|"graph_segments": [^]]*]\|"native_replay": [a-z]*\|"final_loss": [0-9.]*' $O/python.jsonl | tr '\n' ' '; echo
