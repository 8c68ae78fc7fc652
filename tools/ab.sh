# usage: bash tools/ab.sh TAG — bench + kernel stats for tools/ab/libA.so and libB.so on the same box
set -e
R=$GRAFT_REPO_ROOT; T=${1:-x}
cd $R
for v in ${VARIANTS:-A B}; do
  SPWGNN_LIB=$R/${AB_DIR:-tools/ab}/lib$v.so timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab_${T}_$v.json 2> gpurun_out/ab_${T}_$v.err
  echo "$v $(python3 -c "import json;d=json.load(open('gpurun_out/ab_${T}_$v.json'));print(d['value'], d['ms_per_step'])")"
done
cd /tmp && export TMPDIR=/tmp
for v in ${VARIANTS:-A B}; do
  SPWGNN_LIB=$R/${AB_DIR:-tools/ab}/lib$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ab_${T}_prof$v -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-f32-leg > $R/gpurun_out/ab_${T}_prof$v.log 2>&1
done
cd $R
for v in ${VARIANTS:-A B}; do echo "== $v"; python3 tools/profsum.py gpurun_out/ab_${T}_prof$v | head -14; done
