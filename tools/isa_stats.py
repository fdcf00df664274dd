"""Instruction mix of one kernel in a HIP source (offline, gfx950): hipcc --save-temps, then counts of
VALU / SALU / LDS / global instructions and SGPR-spill traffic (v_readlane / v_writelane).

python tools/isa_stats.py smart-quantization_amd/csrc/smaq_pack.hip <kernel-symbol-regex>
"""

import collections
import glob
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    src, pat = sys.argv[1], sys.argv[2]
    tmp = tempfile.mkdtemp()
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17",
                    "-ffp-contract=off", f"-I{REPO}/include", f"-I{REPO}/smart-quantization_amd/csrc",
                    "--save-temps", "-c", os.path.abspath(src), "-o", os.path.join(tmp, "k.o")],
                   cwd=tmp, check=True, stderr=subprocess.DEVNULL)
    s = open(glob.glob(os.path.join(tmp, "*gfx950.s"))[0]).read()
    for m in re.finditer(r"^(" + pat + r"):", s, re.M):
        end = s.index(".Lfunc_end", m.end())
        ins = [l.strip() for l in s[m.end():end].splitlines()
               if l.strip() and not l.strip().startswith((".", ";")) and not l.strip().endswith(":")]
        c = collections.Counter(i.split()[0] for i in ins)
        grp = lambda p: sum(v for k, v in c.items() if k.startswith(p))
        print(m.group(1)[:100])
        print(f"  total {len(ins)} valu {grp('v_')} salu {grp('s_')} ds {grp('ds_')} "
              f"global {grp('global_') + grp('buffer_')} readlane {c['v_readlane_b32']} "
              f"writelane {c['v_writelane_b32']} cndmask {grp('v_cndmask')} mov {grp('v_mov')} "
              f"saveexec {grp('s_and_saveexec')}")
        if len(sys.argv) > 3:
            print("  ", c.most_common(int(sys.argv[3])))


if __name__ == "__main__":
    main()
