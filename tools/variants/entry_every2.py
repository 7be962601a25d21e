# variant: BLAS entries only in every second leaf phase (walk_sim LOCKSTEP
# "... E=2"): a lane standing at an instance leaf waits one iteration when
# the phase is odd, so entry phases gather twice the lanes
import sys
p = sys.argv[1] + "/pt_kernels.hip"
s = open(p).read()
a = """    for(;;)
    {
        if(cursor < end)
        {
            const unsigned long long idle = __ballot(!active);"""
assert s.count(a) == 1
s = s.replace(a, """    uint32_t wave_iter = 0;
    for(;;)
    {
        ++wave_iter;
        if(cursor < end)
        {
            const unsigned long long idle = __ballot(!active);""")
a = "        if(active && w.wants_leaf())\n"
assert s.count(a) == 1
s = s.replace(a, "        if(active && w.wants_leaf() && ((wave_iter & 1u) == 0u || !(w.axis < 0 && w.pend == kBePop)))\n")
open(p, "w").write(s)
