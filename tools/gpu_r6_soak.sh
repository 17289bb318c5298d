#!/bin/bash
# Round 6 soak of the final tree (gpurun): a long headline run (lock-free slot allocation, eventcount
# pool, atomic task groups under sustained load) and a CLI --repeat run whose every pass rewrites and
# re-checks the cohort. → gpurun_out/r6_soak/
set -o pipefail
O=gpurun_out/r6_soak
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u bench.py --steps ${STEPS:-40000} --warmup 5 --no-secondary --wipe-passes 0 --single-passes 0 \
  --cli-runs 0 --keep-data > $O/bench_soak.json 2> $O/bench_soak.err || exit 1
tail -1 $O/bench_soak.json | cut -c1-300
C=/dev/shm/nm03_soak_cohort
build/bin/nm03_synth --data-root $C/ --threads 16 > /dev/null || exit 2
timeout -k 10 300 build/bin/img_processing_parallel --data-root $C/ --out /dev/shm/soak_out --quiet --repeat ${REPEAT:-400} \
  --json $O/cli_repeat.json > $O/cli_repeat.log 2>&1 || exit 3
python3 -c "import json; j=json.load(open('$O/cli_repeat.json')); print('cli repeat: slices', j['slices'], 'ok', j['slices_ok'], 'wall', j.get('wall_s'))"
rm -rf $C /dev/shm/soak_out /dev/shm/nm03_bench_data /dev/shm/nm03_bench_out
echo done
