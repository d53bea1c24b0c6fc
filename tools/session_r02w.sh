# round-2 session: convolution parity incl. S = 4 / 5 on the block tiles (bands compared with the
# same kernel's whole-image build)
exec tools/gpu_session.sh \
  "conv_s45_r02w|600|python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 500 --timeout-method thread -k 'convolution or conv_row_bands'"
