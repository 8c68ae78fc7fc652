set -e
R=$GRAFT_REPO_ROOT; cd $R
for c in ${CS:-0 1 2}; do bash tools/config_artifacts.sh $c r05; done
