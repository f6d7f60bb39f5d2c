# Lab edit: SpMV grid [chunks][bins] instead of [bins][chunks] (speed only; the headline's
# 8 slices and an 8-multiple chunk part keep every block on the same XCD).
s = open('tpl_kcommon.h').read()
a = '''  const int b = blockIdx.x;
  if (b < A.n_slice_blocks) {'''
assert a in s
s = s.replace(a, '''  const int nchb = (int)gridDim.x - A.n_slice_blocks;
  if ((int)blockIdx.x >= nchb) {
    const int b = (int)blockIdx.x - nchb;''')
a = '''  const int chunk = chunk_of_block(A, b - A.n_slice_blocks);'''
assert a in s
s = s.replace(a, '''  const int chunk = chunk_of_block(A, (int)blockIdx.x);''')
open('tpl_kcommon.h', 'w').write(s)
