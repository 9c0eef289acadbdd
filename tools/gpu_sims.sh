# The simulator counterpart on the GPU solvers: C1, C2 and the
# Fig-9 64-GPU run.   gpurun --timeout 600 -- bash tools/gpu_sims.sh <tag>
set -o pipefail
TAG=${1:-sims}
O=gpurun_out/$TAG; mkdir -p $O
T120="120_0.2_5_100_40_25_0,0.5,0.5_0.6,0.3,0.09,0.01_multigpu_dynamic.trace"
T220="220_0.2_5_100_25_4_0,0.5,0.5_0.6,0.3,0.09,0.01_multigpu_dynamic.trace"
timeout -k 10 200 python -u tools/sim_parity.py --trace "$T120" --gpus 32 --max-jobs 50 --solver gpu --out $O/gpu_sim_c1_32.json > $O/c1.log 2>&1 &&
timeout -k 10 200 python -u tools/sim_parity.py --trace "$T120" --gpus 64 --solver gpu --out $O/gpu_sim_c2_64.json > $O/c2.log 2>&1 &&
timeout -k 10 200 python -u tools/sim_parity.py --trace "$T220" --gpus 64 --solver gpu --out $O/gpu_sim_fig9_64.json > $O/fig9.log 2>&1
