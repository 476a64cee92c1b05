# Diagnostic variant: s_sleep(1) before each qmc re-poll round trip
import sys
p = sys.argv[1]; s = open(p).read()
old = """        _Pragma("unroll") for (int kk = 0; kk < QMC_KMAX; ++kk)                              \\
          if (kk < K && (unsigned)(gr[kk] >> 32) != tag)                                     \\"""
new = """        __builtin_amdgcn_s_sleep(1);                                                         \\
        _Pragma("unroll") for (int kk = 0; kk < QMC_KMAX; ++kk)                              \\
          if (kk < K && (unsigned)(gr[kk] >> 32) != tag)                                     \\"""
assert s.count(old) == 1, s.count(old)
s = s.replace(old, new)
open(p, 'w').write(s)
