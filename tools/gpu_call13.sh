# round 4 call 13: seed spread, float64 (two 50 000-iteration lqr_d20 runs sharing the GPU)
bash tools/seed_spread.sh "gpu64:101 gpu64:202"
