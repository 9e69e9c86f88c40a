source tools/gpu_steps.sh
rm -f gpurun_out/steps.log
for c in ekn_d20 lqr_var_d20 vdp_d20; do
  run 1000 tc_$c python tests/train_check.py --config $c --iters 30 --log-freq 10 --runs gpu32,gpu64,oracle --out gpurun_out/train_check_$c.json
done
