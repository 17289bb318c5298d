set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
D=/dev/shm/nm03_cli_data
build/bin/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 1
for r in 1 2 3; do
(cd /tmp && NM03_LOG=info timeout -k 10 60 $GRAFT_REPO_ROOT/build/bin/img_processing_parallel --data-root $D/ --out /dev/shm/nm03_cli_out --json /tmp/cli.json --quiet 2>&1 | grep -E "engine on|set-up" >> $GRAFT_REPO_ROOT/gpurun_out/ctor_cli.txt) || exit 3
python3 -c "import json; d=json.load(open('/tmp/cli.json')); print({k: d[k] for k in ('hip_init_s','engine_ctor_s','engine_setup_s','processing_wall_s')})" >> gpurun_out/ctor_cli.txt
done
