# variant: the wavefront walks read the block order tables from global
# memory (L1 / L2) instead of their LDS copy - no LDS for the table
import sys
p = sys.argv[1] + "/pt_kernels.hip"
s = open(p).read()
a = s.index("    {   // the block order tables (kOrderTables x 8 bytes) after the stack")
b = s.index("    }", s.index("w.lut.p = (const LdsOrderLut::lds_u8_t*)", a)) + len("    }")
s = s[:a] + "    w.lut.p = sc.order_lut;" + s[b:]
s = s.replace("BlockWalker<LdsCold, WalkStack, LdsOrderLut> w;", "BlockWalker<LdsCold, WalkStack, GlobalOrderLut> w;")
s = s.replace("WalkStackOf<false>::type::kLaneBytes) + kOrderTables * 8u", "WalkStackOf<false>::type::kLaneBytes)")
s = s.replace("WalkStackOf<true>::type::kLaneBytes) + kOrderTables * 8u", "WalkStackOf<true>::type::kLaneBytes)")
open(p, "w").write(s)
