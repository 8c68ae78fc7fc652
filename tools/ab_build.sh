# usage: bash tools/ab_build.sh REF — libA.so from git REF (stash round trip), libB.so from the working tree
set -e
mkdir -p ${AB_DIR:-tools/ab}
cd /root/repo
python3 -c "import sys; sys.path.insert(0,'.'); from spwgnn_amd import build; build.build(force=True)" > /dev/null
cp spwgnn_amd/libspwgnn_hip.so ${AB_DIR:-tools/ab}/libB.so
git stash -q
git checkout -q ${1:-HEAD} -- spwgnn_amd/csrc include 2>/dev/null || true
python3 -c "import sys; sys.path.insert(0,'.'); from spwgnn_amd import build; build.build(force=True)" > /dev/null
cp spwgnn_amd/libspwgnn_hip.so ${AB_DIR:-tools/ab}/libA.so
git checkout -q HEAD -- spwgnn_amd/csrc include
git stash pop -q
python3 -c "import sys; sys.path.insert(0,'.'); from spwgnn_amd import build; build.build(force=True)" > /dev/null
ls -la ${AB_DIR:-tools/ab}/
