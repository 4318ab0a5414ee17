set -u
mkdir -p gpurun_out/diff
for w in 1048576 16777216; do
  timeout -k 10 120 oracle/_ref/stack_tx_ref --mss 1460 --bytes $((1<<30)) --write $w --dump gpurun_out/diff/ref_$w.bin || exit 1
  for i in 1 2; do
    timeout -k 10 120 oracle/_ref/stack_tx_amd --mode capture --mss 1460 --bytes $((1<<30)) --write $w --dump gpurun_out/diff/cap_${w}_$i.bin || exit 1
    python3 tools/stack_tx_diff.py gpurun_out/diff/ref_$w.bin gpurun_out/diff/cap_${w}_$i.bin
  done
done
rm -f gpurun_out/diff/*.bin
