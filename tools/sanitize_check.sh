#!/bin/bash
# Host sanitizer sweep (CPU): ASan+leaks, UBSan and TSan builds of the native code
# (device code unaffected: -Xarch_host), each running the CPU paths — DICOM/JPEG codecs, golden
# model, thread pool (cpu-reference = 8 threads), synthetic writer, MetaImage dumps, and the native
# unit tests (thread pool priorities, loopback collectives across threads, loader read paths), and the
# engine's host-only mode (pool workers with private fd tables and creds, slot threads, queued batches).
set -o pipefail
cd "$(dirname "$0")/.."
D=/tmp/nm03_sanitize_data
build/bin/nm03_synth --data-root $D/ --patients 2 --threads 8 > /dev/null || exit 1
# TSan runs the shipping configuration (pool workers with private fd tables and creds): the one
# report that configuration produces — fd numbers reused across private tables — is suppressed by
# tools/tsan.supp, scoped to close() frames.
export ASAN_OPTIONS=detect_leaks=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
export TSAN_OPTIONS="halt_on_error=1 print_suppressions=1 suppressions=$PWD/tools/tsan.supp"
for s in address undefined thread; do
  python build.py --sanitize $s > /tmp/nm03_build_$s.log 2>&1 || { echo "$s: build failed"; exit 2; }
  B=build-$s/bin
  timeout 600 $B/nm03_unit_tests > /tmp/nm03_san_$s.log 2>&1 &&
  timeout 600 $B/test_pipeline --cpu --data-root $D/ --out /tmp/nm03_san_$s/t --dump-mhd /tmp/nm03_san_$s/m >> /tmp/nm03_san_$s.log 2>&1 &&
  timeout 600 $B/nm03_bench --config cpu-reference --data-root $D/ --out /tmp/nm03_san_$s/c --steps 1 --warmup 0 --threads 8 >> /tmp/nm03_san_$s.log 2>&1 &&
  timeout 600 $B/nm03_synth --data-root /tmp/nm03_san_$s/synth/ --patients 2 --threads 4 >> /tmp/nm03_san_$s.log 2>&1 &&
  timeout 900 $B/nm03_bench --config cohort --host-only --data-root $D/ --out /tmp/nm03_san_$s/h --steps 2 --warmup 1 \
    --threads 8 --streams 3 --batch-size 8 >> /tmp/nm03_san_$s.log 2>&1
  rc=$?
  n=$(grep -cE "ERROR: AddressSanitizer|runtime error|WARNING: ThreadSanitizer|LeakSanitizer" /tmp/nm03_san_$s.log)
  echo "$s: rc=$rc reports=$n"
done
