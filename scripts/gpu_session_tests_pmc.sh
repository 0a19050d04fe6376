set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_tests.sh tests/test_gpu_host_paths.py tests/test_gpu_frames.py || exit 1
bash scripts/pmc_work.sh test1 3840 2160 && bash scripts/pmc_work.sh synth1024 3840 2160
