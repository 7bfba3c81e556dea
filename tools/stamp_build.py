"""Builds build/diag/lib_st.so: the library with a stamped copy of csrc/engine_h3.hip (s_memtime at
kernel entry, end of prologue, end of main loop, γ stage 0 landed, pass-0 contraction done, pass-0
outputs done, γ stage 2 landed, pass-1 contraction done, end; wave 0 of each workgroup into a
device array read back by diag_stamps) for tools/h3_stamps.py. Diagnostic build only: the product
library carries no stamps."""
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
C = os.path.join(REPO, "iclr_17_compression_amd", "csrc")
D = os.path.join(REPO, "build", "diag")
os.makedirs(D, exist_ok=True)
s = open(os.path.join(C, "engine_h3.hip")).read()
s = s.replace('#include "common.h"', f'#include "{C}/common.h"').replace('#include "k5_common.h"', f'#include "{C}/k5_common.h"')


def rep(a, b):
    global s
    assert s.count(a) == 1, a[:60]
    s = s.replace(a, b)


rep('''__device__ __attribute__((aligned(16))) unsigned g_zero16h[4] = {0u, 0u, 0u, 0u};''',
    '''__device__ __attribute__((aligned(16))) unsigned g_zero16h[4] = {0u, 0u, 0u, 0u};
__device__ unsigned long long g_st[4096][16];
#define STAMP(i) do { if (threadIdx.x == 0) g_st[blockIdx.x & 4095][i] = __builtin_amdgcn_s_memtime(); } while (0)''')
rep('''  Frag cur;
  int stage = 1;''', '''  STAMP(1);
  Frag cur;
  int stage = 1;''')
rep('''  vm_barrier();   // trailing sink loads landed; every wave is done with the stages''',
    '''  vm_barrier();   // trailing sink loads landed; every wave is done with the stages
  STAMP(2);''')
rep('''  for (int hf = 0; hf < 2; ++hf) {
    // opaque to the optimiser''', '''  for (int hf = 0; hf < 2; ++hf) {
    if (hf) STAMP(5);
    // opaque to the optimiser''')
rep('''        wait_vm_barrier<GK>();   // stage 0 landed (stage 1 in flight)''',
    '''        wait_vm_barrier<GK>();   // stage 0 landed (stage 1 in flight)
        STAMP(3);''')
rep('''        if (q + 1 < 4 && q >= 1) stage_g(q + 1);''', '''        if (q + 1 < 4 && q >= 1) stage_g(q + 1);
        if (q == 2) STAMP(6);''')
rep('''      for (int j = 0; j < 16; ++j) n[il][j] = n[il][j] * nsc;''',
    '''      for (int j = 0; j < 16; ++j) n[il][j] = n[il][j] * nsc;
    STAMP(4 + 3 * hf);''')
rep('''  if (ovf && a.range) atomicOr(a.range, 1);   // vector atomic, per offending lane (rare)
}''', '''  if (ovf && a.range) atomicOr(a.range, 1);   // vector atomic, per offending lane (rare)
  STAMP(8);
  if (threadIdx.x == 0) g_st[blockIdx.x & 4095][10] = __builtin_amdgcn_s_memrealtime();
}''')
rep('''  int bid = blockIdx.x;
  const int per_ph''', '''  STAMP(0);
  if (threadIdx.x == 0) g_st[blockIdx.x & 4095][9] = __builtin_amdgcn_s_memrealtime();
  int bid = blockIdx.x;
  const int per_ph''')
s += '''
extern "C" int diag_stamps(void* dst, long bytes) {
  int r = (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(iclr17::h3k::g_st), bytes, 0, hipMemcpyDeviceToHost);
  static unsigned long long z[4096 * 16];
  hipMemcpyToSymbol(HIP_SYMBOL(iclr17::h3k::g_st), z, sizeof(z), 0, hipMemcpyHostToDevice);
  return r;
}
'''
open(os.path.join(D, "h3d.hip"), "w").write(s)
hipcc = "/opt/rocm/bin/hipcc"
flags = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off"]
subprocess.run([hipcc, *flags, "-c", os.path.join(D, "h3d.hip"), "-o", os.path.join(D, "h3d.o")], check=True)
objs = [os.path.join(C, f) for f in sorted(os.listdir(C)) if f.endswith(".o") and f != "engine_h3.o"]
subprocess.run([hipcc, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", os.path.join(D, "lib_st.so"),
                *objs, os.path.join(D, "h3d.o")], check=True)
os.remove(os.path.join(D, "h3d.o"))
print(os.path.join(D, "lib_st.so"))
