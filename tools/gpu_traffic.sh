#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (separate rocprofv3 runs, --pmc only) per bench config, then
# fold them into profiles/pmc_traffic.json:  bash tools/gpu_traffic.sh 4k zipf open4k 100b zipf@ia8,oa8
# (tokens are tools/pmc_key.py keys: a config plus its non-default layout options)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for key in "$@"; do
  args=$(python3 tools/pmc_key.py args "$key"); f=$(python3 tools/pmc_key.py file "$key")
  for pmc in FETCH_SIZE WRITE_SIZE; do
    echo "== $key $pmc"
    timeout -k 10 240 rocprofv3 --pmc $pmc --output-format csv -d gpurun_out/traffic_${f}_$pmc -o run --kernel-include-regex "k_seal|k_open" -- python3 bench.py --steps 3 --warmup 1 --ramp-ms 0 --no-cpu-baseline --no-roundtrip $args > gpurun_out/traffic_${f}_$pmc.log 2>&1 || { tail -5 gpurun_out/traffic_${f}_$pmc.log; exit 6; }
  done
done
python3 tools/traffic_update.py gpurun_out "$@"
exit 0
