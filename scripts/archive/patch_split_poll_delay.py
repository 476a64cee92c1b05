# Diagnostic variant: the split hand-off (G >= 8) sleeps before its first poll (n s_sleep(1) units)
import sys
p = sys.argv[1]; s = open(p).read()
old = """          poll();
          if (h0 == 0) SP_IMG_WRITE();"""
assert s.count(old) == 1
s = s.replace(old, """          if constexpr (G >= 8) {
            for (int d_ = 0; d_ < 8; ++d_) __builtin_amdgcn_s_sleep(1);
          }
          poll();
          if (h0 == 0) SP_IMG_WRITE();""")
open(p, 'w').write(s)
