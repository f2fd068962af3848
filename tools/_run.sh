timeout -k 10 200 python tools/ab.py --config 4k --knob un0 --values 1 0 --rounds 5 || exit 9
timeout -k 10 200 python tools/ab.py --config open4k --knob un0 --values 1 0 --rounds 5 || exit 9
bash tools/gpu_pmc.sh seal4k_v4 "--config 4k" > gpurun_out/pmc_v4.out 2>&1; tail -16 gpurun_out/pmc_v4.out
