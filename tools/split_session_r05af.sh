# Research A/B (tools/ab/libgdp_exp.so): config 2 with the first / last N tiles of the launch split
# (historical: GDP_SPLIT_HEAD / _TAIL existed only in the research build this A/B measured)
# into two half-width units (GDP_SPLIT_HEAD / GDP_SPLIT_TAIL), v15 and v16 pinned, alternated (round 5)
set -e
mkdir -p gpurun_out
export GDP_LIBRARY=$GRAFT_REPO_ROOT/tools/ab/libgdp_exp.so
for rep in a b; do
  for v in 15 16; do
    for hk in "0 0" "0 256" "0 512" "0 1024" "256 256" "512 0"; do
      set -- $hk
      GDP_SPLIT_HEAD=$1 GDP_SPLIT_TAIL=$2 timeout -k 10 200 python3 bench.py --no-cpu --variant $v --tile-order 0 --zero-window 1 \
        > gpurun_out/split_v${v}_h$1_t$2_${rep}_r05af.log 2>&1
    done
  done
done
echo done
