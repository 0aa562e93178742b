"""Which tail widths break parity on a golden frame (debug helper for seg_finish)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = r'''
import sys, os
sys.path.insert(0, "{root}"); sys.path.insert(0, "{root}/tests")
import numpy as np
import golden_index as GI
import test_gpu_parity as T
gold = GI.load()
for spec in GI.FRAMES:
    land, pose, w, h, aa, ms, ao = GI.unpack(spec)
    if land != "nomadplains":
        continue
    key = GI.frame_key(*spec)
    dev, ter = T.make(GI.consts(w, h, pose), land=land, aa=aa, max_steps=ms, stats=True, ao=ao)
    ter.render_device(); dev.present()
    img = dev.readback_float(); st = dev.stats()
    ref = gold[key + "_rgba32f"]
    bad = ~np.all((img.view(np.uint32) == ref.view(np.uint32)), -1)
    gs = gold[key + "_stats"]
    print(os.environ.get("RT_SEG_LIVE"), key, "bad px", int(bad.sum()), "of", bad.size,
          "noise", st["noise_calls"], gs[0], "prim", st["primary_steps"], gs[2], "sh", st["shadow_steps"], gs[3],
          "ao", st["ao_steps"], gs[6], "hits", st["hits"], gs[5], flush=True)
    if bad.any():
        ys, xs = np.nonzero(bad)
        print("   first bad", list(zip(xs[:8].tolist(), ys[:8].tolist())))
    dev.destroy()
'''
for v in sys.argv[1:] or ["0", "2", "4", "8", "16"]:
    env = dict(os.environ, RT_SEG_LIVE=v)
    r = subprocess.run([sys.executable, "-c", CODE.format(root=ROOT)], env=env, capture_output=True, text=True,
                       timeout=300)
    print(r.stdout, r.stderr[-2000:] if r.returncode else "", flush=True)
    if r.returncode:
        sys.exit(r.returncode)
