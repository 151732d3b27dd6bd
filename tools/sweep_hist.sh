# sweep the device builder's histogram work split (blocks per level) x flush mode
set -o pipefail
timeout -k 10 300 python -m pytest tests/test_gbdt_train.py tests/test_distributed.py -m gpu -q -x 2>&1 | tail -1 || exit 1
for rows in 10500000 1312500; do
  for t in 256 512 1024; do
    for st in 1 0; do
      r=$(YTK_HIST_STAGED=$st YTK_HIST_TARGET=$t timeout -k 10 200 python bench.py --steps 20 --warmup 3 --train-rows $rows --test-rows 62500 2>/dev/null | tail -1 | python -c "import json,sys; d=json.load(sys.stdin); print(d['ms_per_step'], d['train_loss'])") || exit 1
      echo "rows=$rows target=$t staged=$st ms,loss=$r"
    done
  done
done
