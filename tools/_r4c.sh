# per-job weight-gradient times of the SPWGNN_WS_DBG diagnosis builds (ab/libD<n>.so)
cd $GRAFT_REPO_ROOT
for n in 0 1 2 3 4 5 6; do
  SPWGNN_LIB=$GRAFT_REPO_ROOT/ab/libD$n.so timeout -k 10 200 python3 tools/ws_jobs.py 0 2 > gpurun_out/r4c_D$n.txt 2>&1 || { echo "D$n failed"; tail -5 gpurun_out/r4c_D$n.txt; exit 1; }
  echo "D$n $(grep -v '^{' gpurun_out/r4c_D$n.txt | awk '/^(rm|W1|omp|W3|om)/ {printf "%s ", $(NF-6)} /^sum/ {print "sum", $2}')"
done
for n in 0 1 6; do
  SPWGNN_LIB=$GRAFT_REPO_ROOT/ab/libD$n.so timeout -k 10 200 python3 tools/ws_jobs.py 3 2 > gpurun_out/r4c_c3_D$n.txt 2>&1 || { echo "c3 D$n failed"; exit 1; }
  echo "c3 D$n $(grep -v '^{' gpurun_out/r4c_c3_D$n.txt | awk '/^(rm|W1|omp|W3|om)/ {printf "%s ", $(NF-6)} /^sum/ {print "sum", $2}')"
done
