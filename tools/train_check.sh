source tools/gpu_steps.sh
rm -f gpurun_out/steps.log
run 1100 train_check python tests/train_check.py --iters 100 --log-freq 25 --runs gpu32,gpu64,oracle
