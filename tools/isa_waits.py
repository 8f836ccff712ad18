#!/usr/bin/env python3
"""Per kernel of a hipcc --save-temps gfx950 .s file: global loads and full
vmcnt(0) waits (a conditional load in an ILP loop shows up as one wait per
load).  Usage: isa_waits.py <file.s>"""
import re
import sys

s = open(sys.argv[1]).read()
for m in re.finditer(r"^(_Z\w+):[ \t]*;", s, re.M):
    end = s.find("s_endpgm", m.end())
    body = s[m.end():end]
    print(f"{m.group(1)[:70]:70s} loads {body.count('global_load'):4d}  "
          f"vmcnt(0) {body.count('s_waitcnt vmcnt(0)'):4d}")
