"""Build libsmq.so with extra -D flags into exp/<name>/libsmq.so (A/B experiments through SMQ_LIB).
Usage: python tools/build_variant.py <name> -DFLAG[=V] ..."""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as g  # noqa: E402

name, defs = sys.argv[1], sys.argv[2:]
out_dir = os.path.join(g.REPO, "exp", name)
os.makedirs(out_dir, exist_ok=True)
objs, procs = [], []
for src in g.SOURCES:
    obj = os.path.join(out_dir, src.replace(".hip", ".o"))
    objs.append(obj)
    cmd = [g.HIPCC, *g.HIP_FLAGS, *defs, *g.EXTRA_FLAGS.get(src, []), "-c", os.path.join(g.CSRC, src),
           "-o", obj]
    procs.append((cmd, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
for cmd, pr in procs:
    out, _ = pr.communicate()
    if pr.returncode:
        raise SystemExit(out.decode())
subprocess.run([g.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-pthread", "-o",
                os.path.join(out_dir, "libsmq.so"), *objs], check=True)
for o in objs:
    os.remove(o)
print(os.path.join(out_dir, "libsmq.so"))
