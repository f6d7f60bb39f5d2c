# Lab edit: the bins' hand-off without the publish drain. Each slot granule is 8 B:
# {32 bits of the piece sum, 32-bit launch epoch}; the epoch (the row's arrival counter
# / S, read at entry: during a launch it lies in [eS, eS + S - 1] until this publisher
# adds) tags both halves; the last arriver polls the S slots until every tag is this
# launch's epoch. Slots start as all-ones (no epoch matches).
s = open('tpl_device.h').read()
a = '#define TPL_SLOT_STRIDE TPL_MAX_SLICES'
assert a in s
s = s.replace(a, '#define TPL_SLOT_STRIDE (2 * TPL_MAX_SLICES)')
open('tpl_device.h', 'w').write(s)

s = open('tpl_runtime.cpp').read()
a = '''  upload(op, &op->d_P, std::vector<double>(std::max<size_t>(L.lrows.size() * kSlotStride, 1), 0.0));'''
assert a in s
s = s.replace(a, '''  {
    double ones;
    const unsigned long long u = ~0ull;
    std::memcpy(&ones, &u, sizeof ones);
    upload(op, &op->d_P, std::vector<double>(std::max<size_t>(L.lrows.size() * kSlotStride, 1), ones));
  }''')
if '#include <cstring>' not in s:
    s = s.replace('#include <algorithm>', '#include <algorithm>\n#include <cstring>', 1)
open('tpl_runtime.cpp', 'w').write(s)

s = open('tpl_kcommon.h').read()
a = '''  // the finalising thread's own row entries travel with the gathers
  auto pre = epi.pre(sg.row < 0 ? 0 : sg.row);'''
assert a in s
s = s.replace(a, a + '''
  // this publisher's epoch: its row's arrival count before this launch's adds complete
  const unsigned cnt0 = (sg.ri >= 0 && A.n_slices > 1)
      ? __hip_atomic_load(A.Pcnt + (size_t)(sg.ri < 0 ? 0 : sg.ri) * kCntStride, __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_AGENT)
      : 0u;''')
i = s.index('''  unsigned long long* slots = reinterpret_cast<unsigned long long*>(A.P + (size_t)sg.ri * kSlotStride);''')
j = s.index('''  double y = 0.0;
#pragma unroll
  for (int k = 0; k < kSlices; ++k)
    if (k < ns) y = y + __longlong_as_double((long long)v[k]);''')
new = '''  unsigned long long* slots = reinterpret_cast<unsigned long long*>(A.P + (size_t)sg.ri * kSlotStride);
  const unsigned sh = (unsigned)__builtin_ctz((unsigned)ns);
  const unsigned long long ep = (unsigned long long)(cnt0 >> sh) << 32;
  const unsigned long long pb = (unsigned long long)__double_as_longlong(p);
  __hip_atomic_store(slots + 2 * s, (pb & 0xffffffffull) | ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(slots + 2 * s + 1, (pb >> 32) | ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  TPL_MARK(4);
  const unsigned int arrived = __hip_atomic_fetch_add(A.Pcnt + (size_t)sg.ri * kCntStride, 1u,
                                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("" ::: "memory");  // the slot loads stay behind the returned add
  if ((arrived & (unsigned)(ns - 1)) != (unsigned)(ns - 1)) return;
  static_assert(kSlices == 8, "eight slot granule pairs");
  typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
  unsigned long long v[kSlices];
  for (int it = 0; it < (1 << 16); ++it) {
    u64x2 r0, r1, r2, r3, r4, r5, r6, r7;
    asm volatile(
        "global_load_dwordx4 %0, %8, off sc1\\n\\t"
        "global_load_dwordx4 %1, %9, off sc1\\n\\t"
        "global_load_dwordx4 %2, %10, off sc1\\n\\t"
        "global_load_dwordx4 %3, %11, off sc1\\n\\t"
        "global_load_dwordx4 %4, %12, off sc1\\n\\t"
        "global_load_dwordx4 %5, %13, off sc1\\n\\t"
        "global_load_dwordx4 %6, %14, off sc1\\n\\t"
        "global_load_dwordx4 %7, %15, off sc1\\n\\t"
        "s_waitcnt vmcnt(0)"
        : "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3), "=&v"(r4), "=&v"(r5), "=&v"(r6), "=&v"(r7)
        : "v"(slots), "v"(slots + (1 < ns ? 2 : 0)), "v"(slots + (2 < ns ? 4 : 0)),
          "v"(slots + (3 < ns ? 6 : 0)), "v"(slots + (4 < ns ? 8 : 0)), "v"(slots + (5 < ns ? 10 : 0)),
          "v"(slots + (6 < ns ? 12 : 0)), "v"(slots + (7 < ns ? 14 : 0))
        : "memory");
    const u64x2 rr[kSlices] = {r0, r1, r2, r3, r4, r5, r6, r7};
    bool ok = true;
#pragma unroll
    for (int k = 0; k < kSlices; ++k) {
      ok = ok && (rr[k].x >> 32) == (ep >> 32) && (rr[k].y >> 32) == (ep >> 32);
      v[k] = (rr[k].x & 0xffffffffull) | (rr[k].y << 32);
    }
    if (ok) break;
    __builtin_amdgcn_s_sleep(1);
  }
'''
s = s[:i] + new + s[j:]
open('tpl_kcommon.h', 'w').write(s)
