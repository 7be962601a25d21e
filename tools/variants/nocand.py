# variant: no any-hit occluder candidates (the walk as before, with the new code present)
import sys
p = sys.argv[1] + "/pt_kernels.hip"
s = open(p).read()
a = "if(ANY) w.try_candidate(sc, occ_inst, occ_prim, meta_sub(m));"
assert a in s
open(p, "w").write(s.replace(a, ""))
