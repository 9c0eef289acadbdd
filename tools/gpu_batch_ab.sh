# Interleaved C3 bench at 32768 and 65536 instances per step (no legs).
set -o pipefail
O=gpurun_out/batch_ab; mkdir -p $O
for i in 1 2; do
  for b in 32768 65536; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-legs --batch $b > $O/b${b}_$i.json 2> $O/b${b}_$i.err || exit 1
  done
done
python3 -c "
import json,glob
for f in sorted(glob.glob('$O/b*.json')):
    d=json.load(open(f)); print(f, round(d['value']), d['ms_per_step'])"
