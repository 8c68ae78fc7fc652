# usage: bash tools/round_refresh_ab.sh TAG CONFIG... — small-batch A/B + GPU tests (tools/small_ab.sh),
# smoke, then the committed per-config artifacts (tools/config_artifacts.sh) for the given configs
set -e
R=$GRAFT_REPO_ROOT; T=$1; shift
cd $R
bash tools/small_ab.sh
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1
tail -1 gpurun_out/${T}_smoke.log
SKIP_TESTS=1 bash tools/refresh_round.sh $T "$@"
