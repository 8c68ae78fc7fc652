set -e
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 300 python3 tools/bf16_plan_probe.py 6 24 0
timeout -k 10 300 python3 tools/bf16_plan_probe.py 6 20 0
timeout -k 10 300 python3 tools/bf16_plan_probe.py 4 24 1
