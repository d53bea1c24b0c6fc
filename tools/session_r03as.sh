# round-3 session as: store pacing in the in-place re-entry (k_levels MODE 3: five stores per thread)
# — A/B over block shape x zero window x pace on configs 2 / 4 / 5
T="python tools/tune.py --rounds 7"
R="op=regen,sub=8;op=regen,sub=8,sp=0;op=regen,sub=8,sp=1;op=regen,sub=8,zw=1,sp=0;op=regen,sub=16;op=regen,sub=16,sp=0;op=regen,sub=16,sp=1;op=regen,sub=1,zw=1,sp=0;op=regen,sub=4,zw=1,sp=1;op=regen,sub=0,zw=1"
exec tools/gpu_session.sh \
  "spi_regen_c2_r03as|300|$T --config c2 --rotate 5 --iters 10 --variants '$R'" \
  "spi_regen_c4_r03as|400|$T --config c4 --iters 2 --rounds 5 --variants '$R'" \
  "spi_regen_c5_r03as|300|$T --config c5 --iters 2 --variants '$R'"
