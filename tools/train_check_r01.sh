# Training-level parity of the production path (HIP graphs + split steps) against the
# oracle histories already in profiles/ (same seeds, same settings).
source tools/gpu_steps.sh
rm -f gpurun_out/steps.log
run 600 tc_lqr_d20 python -u tests/train_check.py --config lqr_d20 --iters 100 --log-freq 25 --runs gpu32,gpu64 --oracle-from profiles/r01_train_check_lqr_d20.json --out gpurun_out/train_check_lqr_d20.json
for c in ekn_d20 lqr_var_d20 vdp_d20; do
  run 400 tc_$c python -u tests/train_check.py --config $c --iters 30 --log-freq 10 --runs gpu32,gpu64 --oracle-from profiles/r01_train_check_$c.json --out gpurun_out/train_check_$c.json
done
