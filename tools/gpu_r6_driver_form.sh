#!/bin/bash
# Round 6: the driver's exact 1-GPU command (bench.py --gpus 1 --steps 20 --warmup 5, every secondary figure
# included) repeated on one box, to show the spread of a 23 ms timed window. → gpurun_out/r6_driver/
set -o pipefail
O=gpurun_out/r6_driver
mkdir -p $O
export PYTHONUNBUFFERED=1
for r in $(seq ${RUNS:-6}); do
  timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_$r.json 2> $O/bench_$r.err || exit 1
  python3 -c "
import json; j = json.loads(open('$O/bench_$r.json').read().strip().splitlines()[-1]); c = j['config']
print('run $r', j['value'], 'cpu/step', c['rank0_process_cpu_ms_per_step'], 'wipe', c['wipe_each_pass']['value'],
      c['wipe_each_pass']['timed_s'], 'cli median', c['cli_wall']['wall_median_s'])"
done
echo done
