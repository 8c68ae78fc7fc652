# FETCH_SIZE calibration per load width, then the bf16 edge forward's bytes by operand class
# (config 3, -DSPWGNN_DIAG library: SPWGNN_EFWD_DBG 1 = A rows from 8 cached blocks, 3 = U/V rows of
# the tile's first node). usage: bash tools/gpu_r5h.sh
set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $R/gpurun_out/fcal -o run --output-format csv -- $R/tools/bin/fetchcal > $R/gpurun_out/fcal.log 2>&1
B="$R/bench.py --config 3 --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-table --roofline-kernel edge_fwd"
for V in 0 1 3; do
  SPWGNN_LIB=$R/abl/libD.so SPWGNN_EFWD_DBG=$V timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $R/gpurun_out/efA$V -o run --output-format csv -- python3 $B > $R/gpurun_out/efA$V.log 2>&1
  SPWGNN_LIB=$R/abl/libD.so SPWGNN_EFWD_DBG=$V timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $R/gpurun_out/efB$V -o run --output-format csv -- python3 $B > $R/gpurun_out/efB$V.log 2>&1
done
cd $R
python3 - <<'PY'
import csv, collections
def load(d):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f"gpurun_out/{d}/run_counter_collection.csv")):
        acc[(r["Dispatch_Id"], r["Kernel_Name"].split("(")[0].replace("void ", "").replace("spw::", ""))].append(float(r["Counter_Value"]))
    per = collections.defaultdict(list)
    for (disp, k), v in acc.items():
        per[k].append(sum(v))
    return per
cal = load("fcal")
for k, v in cal.items():
    print("calibration", k[:40], [round(x * 1024 / 2**30, 3) for x in v], "× 1 GiB (FETCH_SIZE KiB → GiB; the reads are 1 GiB)")
for V in (0, 1, 3):
    f, w = load(f"efA{V}"), load(f"efB{V}")
    for k in f:
        if "edge_fwd" in k:
            print(f"EFWD_DBG={V} {k[:48]} FETCH {sum(f[k])/len(f[k])*1024/1e9:.3f} GB/launch (raw, uncorrected)  WRITE {sum(w[k])/len(w[k])*1024/1e9:.3f} GB/launch")
PY
