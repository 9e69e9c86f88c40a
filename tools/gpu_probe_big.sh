source tools/gpu_steps.sh
export TMPDIR=/tmp
rm -f gpurun_out/steps.log
run 200 probe_nn_big python -u tools/probe_nn.py --B 2048,8192,16384 --N 100 --reps 3
run 200 probe_nn_big_save python -u tools/probe_nn.py --B 2048,8192,16384 --N 100 --reps 3 --save
