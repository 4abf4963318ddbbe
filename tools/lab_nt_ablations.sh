set -u
for m in 0 1 2 4 8 5; do
  TAG=lab_nt LAB_TIMEOUT=90 bash tools/run_lab.sh tools/b3_lab_m$m > /dev/null 2>&1 || { echo "m$m failed rc=$?"; exit 1; }
  echo "== m$m"; grep -E "^b3 |^f32" gpurun_out/lab_nt/b3_lab_m$m.txt
done
