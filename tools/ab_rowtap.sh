#!/usr/bin/env bash
# round 3: A/B of the row-window layout of non-square images (GDP_ROWTAP_LAYOUT 0 = [scale][row],
# 1 = [row][scale]), alternated twice, with image-0 checksums for the bit-exactness comparison:
# the tall 65536 x 4096 image, config 3 (64 x 1080 x 1920) build and re-entry.
for rep in 1 2; do
  for lay in 0 1; do
    for spec in "c2|--shape 65536x4096x1|v=15;v=16;v=0;v=15,ord=1|build" "c2|--shape 16384x4096x1 --rotate 2|v=15;v=16;v=0|build" \
                "c3||v=11;v=17;v=15;v=11,ord=1|build" "c3||sub=1;sub=4;sub=2|regen" "c2|--shape 65536x4096x1|sub=1;sub=4|regen"; do
      IFS='|' read -r cfg extra vars op <<< "$spec"
      its=20
      echo "## rep $rep layout $lay cfg $cfg $extra op $op"
      GDP_ROWTAP_LAYOUT=$lay timeout -k 10 150 python tools/tune.py --config $cfg $extra --iters $its --rounds 5 --no-check \
         --checksums --op $op --variants "$vars" 2>&1 | grep variant || exit 1
    done
  done
done
