# variant: the any-hit walk's run length (consecutive queue groups per wave run), env PTG_RUN
import os
import sys
p = sys.argv[1] + "/pt_kernels.hip"
s = open(p).read()
a = "#define PTG_ANY_RUN 4\n"
assert a in s
open(p, "w").write(s.replace(a, "#define PTG_ANY_RUN %d\n" % int(os.environ["PTG_RUN"])))
