set -u
bash scripts/sq_passes.sh r05ah_c3 --steps 2 --warmup 1 --no-roofline --cpu-sample 0 && python scripts/sq_ratios.py gpurun_out/pmc_r05ah_c3 --top 24 > gpurun_out/r05ah_sq_ratios_c3.md && bash scripts/sq_passes.sh r05ah_c5 --config 5 --steps 2 --warmup 1 --no-roofline --cpu-sample 0 && python scripts/sq_ratios.py gpurun_out/pmc_r05ah_c5 --top 24 > gpurun_out/r05ah_sq_ratios_c5.md
