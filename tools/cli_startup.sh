#!/bin/bash
# (gpurun) where the CLI wall clock goes: bare HIP runtime init, then img_processing_parallel on the
# full cohort (wall vs HIP init, engine construction and processing from --json) with the fast
# CLI exit on and off (NM03_FAST_EXIT), interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/cli_startup.txt
: > $O
D=/dev/shm/nm03_cli_data
build/bin/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 1
for r in 1 2 3 4; do
  python3 - >> $O <<'PY' || exit 2
import ctypes, time
t0 = time.perf_counter()
lib = ctypes.CDLL("libamdhip64.so")
t1 = time.perf_counter()
n = ctypes.c_int()
lib.hipGetDeviceCount(ctypes.byref(n))
lib.hipSetDevice(0)
p = ctypes.c_void_p()
lib.hipMalloc(ctypes.byref(p), 1 << 20)
lib.hipDeviceSynchronize()
t2 = time.perf_counter()
print(f"hip: dlopen {1e3*(t1-t0):.1f} ms, init+first malloc {1e3*(t2-t1):.1f} ms")
PY
done
for r in 1 2 3 4 5 6; do
  for fx in 1 0; do
    s=$(date +%s.%N)
    (cd /tmp && NM03_FAST_EXIT=$fx timeout -k 10 60 $GRAFT_REPO_ROOT/build/bin/img_processing_parallel --data-root $D/ --out /dev/shm/nm03_cli_out --json /tmp/cli.json --quiet > /dev/null 2>&1) || exit 3
    e=$(date +%s.%N)
    python3 -c "
import json
d = json.load(open('/tmp/cli.json'))
w = ($e - $s) * 1e3
print(f'[fast_exit={$fx}] cli wall {w:.1f} ms; hip_init {1e3*d[\"hip_init_s\"]:.1f} ms, engine_ctor {1e3*d[\"engine_ctor_s\"]:.1f} ms, '
      f'setup {1e3*d[\"engine_setup_s\"]:.1f} ms, processing {1e3*d[\"processing_wall_s\"]:.1f} ms, '
      f'rest {w - 1e3*(d[\"engine_setup_s\"] + d[\"processing_wall_s\"]):.1f} ms')" >> $O || exit 4
  done
done
rm -rf $D /dev/shm/nm03_cli_out
