# Lab edit: bins dispatched in a rotated order (m -> (m + 36) mod M; speed only): the
# heaviest bins (m = 64..67 at 500k) no longer share CU classes 0..3 with m = 0..3.
s = open('tpl_kcommon.h').read()
a = '''      s = T * (b & 7) + q % T;
      m = q / T;'''
assert a in s
s = s.replace(a, '''      s = T * (b & 7) + q % T;
      const int Mb = A.n_slice_blocks / A.n_slices;
      m = (q / T + 36) % Mb;''')
open('tpl_kcommon.h', 'w').write(s)
