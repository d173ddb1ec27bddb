"""Run tools/colbench.py once per environment variant (fresh process each: the engine reads its
RQHIP_* knobs once).  usage: python tools/sweep.py OUT.log 'JSON list of env dicts' [colbench args]"""
import json
import os
import subprocess
import sys

out, variants = sys.argv[1], json.loads(sys.argv[2])
args = sys.argv[3:] or ["1024", "1200", "1100", "1024", "10"]
with open(out, "w") as f:
    for v in variants:
        f.write("== %s\n" % json.dumps(v))
        f.flush()
        env = dict(os.environ, **v)
        r = subprocess.run([sys.executable, "-u", "tools/colbench.py"] + args, env=env, stdout=f,
                           stderr=subprocess.STDOUT, timeout=150)
        if r.returncode != 0:
            f.write("rc=%d\n" % r.returncode)
            sys.exit(3)
