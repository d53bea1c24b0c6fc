# round-2 session: EXPERIMENT — the build's last N units store write-through (nt sc1, line not
# kept in L2) so the end-of-kernel L2 write-back has less dirty data; bits first, then cold A/B
V="v=15;v=15,wt=128;v=15,wt=256;v=15,wt=512;v=15,wt=1024;v=15,wt=2048"
exec tools/gpu_session.sh \
  "wt_check_r02am|200|python3 tools/wt_check.py" \
  "ab_wt_c2_r02am|240|python3 tools/tune.py --config c2 --rotate 5 --iters 20 --rounds 11 --variants '$V'" \
  "ab_wt_c5_r02am|240|python3 tools/tune.py --config c5 --iters 5 --rounds 7 --variants 'v=15;v=15,wt=512;v=15,wt=1024;v=15,wt=4096'" \
  "ab_wt_c4_r02am|300|python3 tools/tune.py --config c4 --iters 3 --rounds 5 --variants 'v=15,ord=1;v=15,ord=1,wt=512;v=15,ord=1,wt=1024;v=15,ord=1,wt=4096'"
