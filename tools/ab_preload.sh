#!/usr/bin/env bash
# round 3: A/B of PATH 3 with the windows / input preloaded ahead of the first store
# (GDP_PRELOAD 1: row windows, 2: + column windows, 3: + the input pixel) against the shipped
# build, alternated twice, on the tall non-square image, configs 2-5.
# Checksums of image 0 per variant/library for the bit-exactness comparison.
L=sift-parallel-optimization_amd/lib
for rep in 1 2; do
  for lib in $L/libgdp.so $L/libgdp_pre1.so $L/libgdp_pre2.so $L/libgdp_pre3.so; do
    for spec in "c2|--rotate 5|v=15;v=16;v=15,ord=1" "c2|--shape 65536x4096x1|v=15;v=16;v=18;v=15,ord=1;v=0" \
                "c3||v=11;v=17;v=16;v=17,ord=1" "c4||v=15;v=15,ord=1" "c5||v=15;v=15,ord=1"; do
      cfg="${spec%%|*}"; rest="${spec#*|}"; extra="${rest%%|*}"; vars="${rest#*|}"
      its=20; [ "$cfg" = c2 ] && its=50
      echo "## rep $rep lib $lib cfg $cfg $extra"
      GDP_LIBRARY=$lib timeout -k 10 150 python tools/tune.py --config $cfg $extra --iters $its --rounds 5 --no-check \
         --checksums --variants "$vars" 2>&1 | grep variant || exit 1
    done
  done
done
