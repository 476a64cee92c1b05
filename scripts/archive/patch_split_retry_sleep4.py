# Diagnostic variant: the split hand-off sleeps s_sleep(4) (not 1) before each re-poll
import sys
p = sys.argv[1]; s = open(p).read()
old = """            __builtin_amdgcn_s_sleep(1);
            poll();"""
assert s.count(old) == 1
s = s.replace(old, """            __builtin_amdgcn_s_sleep(4);
            poll();""")
open(p, 'w').write(s)
