"""Incremental build of libsmq.so for development (objects kept in build/obj; a source is recompiled
when it or any header under csrc/ or include/ is newer than its object). build() in
__graft_entry__.py stays the one-shot full build the driver runs.  python tools/ibuild.py"""

import glob
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import __graft_entry__ as G  # noqa: E402

OBJ = os.path.join(REPO, "build", "obj")
os.makedirs(OBJ, exist_ok=True)
headers = glob.glob(os.path.join(G.CSRC, "*.h")) + glob.glob(os.path.join(REPO, "include", "*.h"))
hmax = max(os.path.getmtime(h) for h in headers)
procs, objs = [], []
for src in G.SOURCES:
    sp = os.path.join(G.CSRC, src)
    obj = os.path.join(OBJ, src.replace(".hip", ".o"))
    objs.append(obj)
    if os.path.exists(obj) and os.path.getmtime(obj) >= max(hmax, os.path.getmtime(sp)):
        continue
    cmd = [G.HIPCC, *G.HIP_FLAGS, *G.EXTRA_FLAGS.get(src, []), "-c", sp, "-o", obj]
    print("hipcc", src, flush=True)
    procs.append((cmd, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
for cmd, pr in procs:
    out, _ = pr.communicate()
    if pr.returncode:
        sys.exit(f"hipcc failed: {' '.join(cmd)}\n{out.decode()}")
# linked next to the library, then renamed over it: a reader (a gpurun upload) sees the old or the
# new file, never a partial one
tmp = G.LIB + ".tmp"
link = [G.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-pthread", "-o", tmp, *objs]
r = subprocess.run(link, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
if r.returncode:
    sys.exit(f"link failed\n{r.stdout.decode()}")
os.replace(tmp, G.LIB)
print("linked", G.LIB)
