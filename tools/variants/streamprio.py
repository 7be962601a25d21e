# variant: stream priorities - the chunk pipelines' main streams (camera,
# closest-hit walk, classify, shade: the critical path) created at the
# greatest priority (SIDE=1: the side streams instead)
import os, sys
p = sys.argv[1] + "/pt_kernels.hip"
s = open(p).read()
which = "b.side" if os.environ.get("SIDE") == "1" else "b.main"
a = "        PTG_HIP(hipStreamCreateWithFlags(&%s, hipStreamNonBlocking));\n" % which
assert a in s
s = s.replace(a, """        {
            int least = 0, greatest = 0;
            PTG_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
            PTG_HIP(hipStreamCreateWithPriority(&%s, hipStreamNonBlocking, greatest));
        }
""" % which)
open(p, "w").write(s)
