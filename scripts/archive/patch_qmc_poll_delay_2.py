# Diagnostic variant: s_sleep(2) between the qmc publish and its first poll
import sys
p = sys.argv[1]; s = open(p).read()
old = """      unsigned long long gr[QMC_KMAX];                                                       \\
      _Pragma("unroll") for (int kk = 0; kk < QMC_KMAX; ++kk)                                \\
        if (kk < K) gr[kk] = __hip_atomic_load("""
new = """      unsigned long long gr[QMC_KMAX];                                                       \\
      __builtin_amdgcn_s_sleep(2);                                                          \\
      _Pragma("unroll") for (int kk = 0; kk < QMC_KMAX; ++kk)                                \\
        if (kk < K) gr[kk] = __hip_atomic_load("""
assert s.count(old) == 1, s.count(old)
s = s.replace(old, new)
open(p, 'w').write(s)
