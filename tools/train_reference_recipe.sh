#!/bin/bash
# The reference's own training recipe for the bench shape (scripts/Synthetic.sh:3: QP_1000_500_500,
# outer_T = truncated_length = 100, hidden 800, lr 5e-5, batch 2, data_size 1000, eq/ineq tol 0.2,
# EarlyStopping on the validation violations, configs/QP.yaml for the rest) through this repo's
# main.py train mode, on synthetic instances with seeds 100017 + i (disjoint from the bench's
# 17 + i), for at most <minutes> of wall time per call, continuing from the state file of the
# previous call (main.py --resume; each call ends after the epoch that crosses <minutes>); then the
# K = 100 residual of whatever EarlyStopping saved, on the bench's 1024 instances.  The state file and
# checkpoint live under checkpoints/recipe_<tag>/ so that they travel with the tree to the next call.
# Usage: bash tools/train_reference_recipe.sh <tag> <minutes>
set -o pipefail
tag=${1:-r03}; mins=${2:-20}
out=gpurun_out/${tag}_recipe
st=checkpoints/recipe_${tag}
mkdir -p "$out" "$st"
timeout -k 10 $(( (${mins%.*} + 8) * 60 )) python3 -u main.py --config ./configs/QP.yaml --model_name LSTM --prob_type QP \
  --outer_T 100 --truncated_length 100 --hidden_dim 800 --eq_tol 0.2 --ineq_tol 0.2 --num_var 1000 --num_ineq 500 \
  --num_eq 500 --input_dim 2 --data_size 1000 --batch_size 2 --lr 0.00005 --scaling \
  --synthetic --seed 100017 --save_dir "$st/results" --resume "$st/resume.pt" --max_minutes "$mins" \
  >> "$out/train.log" 2>> "$out/train.err"
rc=$?
cp -r "$st" "$out/"  # brought back to the builder (gpurun_out is what returns)
echo "train rc=$rc"
ck="$st/results/lstm/params/QP_1000_500_500_100_800.pth"
if [ $rc -eq 0 ] && [ -f "$ck" ]; then
  timeout -k 10 300 python3 -u bench.py --weights "$ck" --steps 1 --warmup 0 --cpu-sample 0 --stage2-iters 0 \
    --alt-f16x3 0 --train-batch 0 > "$out/bench_recipe.json" 2> "$out/bench_recipe.err"
  echo "bench rc=$?"
else
  echo "no checkpoint saved by EarlyStopping"
fi
