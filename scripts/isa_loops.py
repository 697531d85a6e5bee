"""Loop-level instruction mix of one kernel in a gfx950 ISA listing:
python3 scripts/isa_loops.py build/gqmap_engine.s <mangled-kernel-name>"""
import re
import sys

txt = open(sys.argv[1]).read()
name = sys.argv[2]
s = txt.find(name + ": ")
if s < 0:
    s = txt.find(name + ":\n")
e = txt.find(".Lfunc_end", s)
body = txt[s:e].split("\n")
labels = {}
for i, l in enumerate(body):
    m = re.match(r"^(\.LBB\S+):", l)
    if m:
        labels[m.group(1)] = i
loops = []
for i, l in enumerate(body):
    m = re.search(r"s_cbranch_\w+\s+(\.LBB\S+)|s_branch\s+(\.LBB\S+)", l)
    if m:
        t = m.group(1) or m.group(2)
        if t in labels and labels[t] < i:
            loops.append((labels[t], i))


def mix(seg):
    c = lambda f: sum(1 for x in seg if f(x))
    return dict(valu=c(lambda x: re.match(r"\s+v_", x) and "lane_b32" not in x),
                f64=c(lambda x: re.match(r"\s+v_\w+_f64", x)),
                cvt=c(lambda x: "v_cvt_f64_f32" in x),
                rsq=c(lambda x: "v_rsq" in x or "v_sqrt" in x),
                lane=c(lambda x: "lane_b32" in x),
                vmem=c(lambda x: "global_load" in x or "buffer_load" in x),
                smem=c(lambda x: "s_load" in x or "s_buffer_load" in x),
                lds=c(lambda x: "ds_" in x),
                scratch=c(lambda x: "scratch_" in x),
                salu=c(lambda x: re.match(r"\s+s_", x) is not None))


print(len(body), "lines; whole kernel:", mix(body))
for a, b in loops:
    print(f"loop {a}-{b} ({b - a} lines):", mix(body[a:b + 1]))
