set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python scripts/multi_probe.py > gpurun_out/multi_probe2.json 2> gpurun_out/multi_probe2.err; cat gpurun_out/multi_probe2.json
bash scripts/gpu_hv_timeline.sh
