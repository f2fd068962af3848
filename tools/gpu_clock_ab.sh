#!/bin/bash
# Clock and time of the 4k seal with and without its HBM traffic (diagnostic builds, see
# CZ_DIAG_* in cz_kernels.hip):  bash tools/gpu_clock_ab.sh lib1.so lib2.so ...
# Per library: the bench's HIP-event kernel time, then one PMC pass (SQ_INSTS_VALU,
# GRBM_GUI_ACTIVE) over a ramped run; tools/clock_summary.py prints the per-dispatch clock.
# CZ_CLOCK_CONFIG=zipf|open4k|100b measures another bench config (default 4k).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
cfg=${CZ_CLOCK_CONFIG:-4k}
rt=""; [ "$cfg" = 4k ] && rt="--no-roundtrip"
for lib in "$@"; do
  tag=${lib%.so}
  CZ_LIB=$PWD/jeromq_amd/$lib timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 10 --no-cpu-baseline $rt --no-verify > gpurun_out/clk_$tag.log 2>&1 || { tail gpurun_out/clk_$tag.log; exit 5; }
  CZ_LIB=$PWD/jeromq_amd/$lib timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/clkpmc_$tag -o run --kernel-include-regex "k_seal|k_open" -- python3 bench.py --config $cfg --steps 20 --warmup 10 --no-cpu-baseline $rt --no-verify > gpurun_out/clkpmc_$tag.log 2>&1 || { tail -5 gpurun_out/clkpmc_$tag.log; exit 6; }
  python3 tools/clock_summary.py gpurun_out $tag $cfg
done
exit 0
