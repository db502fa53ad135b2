"""Generate tools/micro/cemit_bench.hip: the production k_class_emit on a synthetic LUBM-shaped class
(2 classes x 35k members, 71k-entry lists) plus ablation variants (dev tool)."""
import os
import re

here = os.path.dirname(os.path.abspath(__file__))
src = open(os.path.join(here, "..", "..", "rdfind_amd", "csrc", "kernels.inl")).read()
body = re.search(r"__global__ __launch_bounds__\(RDF_BLOCK\) void k_class_emit\(.*?\n}\n", src, re.S).group(0)


def variant(name, nolds=False, nostage=False):
    b = body.replace("void k_class_emit(", f"void {name}(")
    if nolds:
        b = b.replace("val[j] = sl[(q + (q >= skip ? 1 : 0)) & (int)(CLS_LS - 1)];", "val[j] = (u32)(q + (q >= skip ? 1 : 0));")
    if nostage:
        b = b.replace("for (u64 i = threadIdx.x; i < p1 - p0; i += RDF_BLOCK) sl[i] = lists[lb + p0 + i];", "")
    return b


code = ['#include "../../rdfind_amd/csrc/kernels.inl"', "namespace rdf {",
        variant("v_nolds", nolds=True), variant("v_nolds_nostage", nolds=True, nostage=True), "}",
        open(os.path.join(here, "cemit_main.inc")).read()]
open(os.path.join(here, "cemit_bench.hip"), "w").write("\n".join(code))
