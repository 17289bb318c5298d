#!/bin/bash
# (gpurun) Round 4, fifth call. gpurun_out/r4e/:
#  * GPU tests (threaded z-slab rehearsal test, fast exit via on_exit);
#  * nm03_bench under rocprofv3: exit status + kernel stats written (fast exit keeps the profiler's
#    exit handler); JPEG encoder split isolated (variants 0 / 40 gray only / 41 label only / 7 / 1 / 2 / 4 / 15);
#  * z-slab rehearsal in one process (rank threads, loopback comms): 256³ phantom, 1 / 2 / 4 ranks;
#  * default bench (cli_wall, wipe passes with 4 reaper threads).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r4e; mkdir -p $O/split
B=build/bin
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || exit 10
D=/tmp/r4e_data
$B/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 11
for v in 0 40 41 7 1 2 4 15; do
  NM03_PROFILE_VARIANT=jpeg=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/split/v$v -o k \
    -- $B/nm03_bench --config cohort --data-root $D/ --steps 3 --warmup 1 --streams 1 --batch-size 96 \
    > $O/split/v$v.log 2>&1
  echo "v$v exit $?" >> $O/split/status.txt
done
rm -rf $D
timeout -k 10 300 python3 - > $O/slab_threads.txt 2>&1 <<'PY' || exit 20
import sys, time, numpy as np
sys.path.insert(0, ".")
import nm03_capstone_project_amd as nm
n = nm.native()
d = 256
vol = np.stack([n.phantom_slice(256, 256, 3, z % 23, 23, 7) for z in range(d)])
vol[:, 100:140, :] = 1500  # an in-band slab through every plane: boundary exchange every round
ref = n.VolumeRunner(0)
ref.run(vol, n.PipelineParams(), 6, 7, [])
t = []
for _ in range(5):
    t0 = time.perf_counter(); r = ref.run(vol, n.PipelineParams(), 6, 7, []); t.append(time.perf_counter() - t0)
print(f"single VolumeRunner.run (incl. mask read-back): median {1e3*sorted(t)[2]:.2f} ms, kernels {1e3*r['kernels_s']:.2f} ms")
for k in (1, 2, 4):
    s = n.run_volume_slabs_threads(vol, k, n.PipelineParams(), 6, 7, 0, 7)
    ok = np.array_equal(s["region"], r["region"]) and np.array_equal(s["dilated"], r["dilated"])
    w = sorted(s["walls_s"])
    print(f"{k} rank threads: split wall median {1e3*w[len(w)//2]:.2f} ms min {1e3*w[0]:.2f} ms, rounds {s['rounds']}, "
          f"exchanged {s['exchanged_bytes']}, identical {ok}")
PY
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 30
