"""rocprofv3 kernel symbol -> athd profile label (prof.h): drop 'void ', 'athd::', the argument list, spaces and
the 'u' suffix of unsigned template arguments.  e.g. 'void athd::gemm3_kernel<256, 192, 4, 2, 2, 200u>(athd::GemmDesc)'
-> 'gemm3_kernel<256,192,4,2,2,200>'."""
import re


def short_name(sym: str) -> str:
    s = sym.strip()
    if s.startswith("void "):
        s = s[5:]
    s = s.replace("athd::", "")
    depth, cut = 0, len(s)
    for i, ch in enumerate(s):       # the argument list is the first '(' outside template brackets
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            cut = i
            break
    s = s[:cut].replace(" ", "")
    return re.sub(r"(\d+)u\b", r"\1", s)
