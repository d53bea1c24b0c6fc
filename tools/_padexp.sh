for pad in 0 16777216 50000000 134217728; do
  for shape in 65536x4096x1; do
    echo "pad=$pad shape=$shape"
    GDP_LEVEL_PAD=$pad timeout -k 10 120 python tools/tune.py --shape $shape --iters 10 --rounds 3 --variants "v=0;v=0,ord=1" 2>&1 | grep variant || exit 1
  done
done
