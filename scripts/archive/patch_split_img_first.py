# Diagnostic variant: the split hand-off writes the slice image BEFORE its first poll (the
# image write then delays the poll instead of running while it is in flight)
import sys
p = sys.argv[1]; s = open(p).read()
old = """          poll();
          if (h0 == 0) SP_IMG_WRITE();"""
assert s.count(old) == 1
s = s.replace(old, """          if (h0 == 0) SP_IMG_WRITE();
          poll();""")
open(p, 'w').write(s)
