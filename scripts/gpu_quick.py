import sys, time, os
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests')
import numpy as np
import gpgpuraytrace_amd as G
import oracle_lib as O
W, H = 96, 64
nz = O.noise_tables()
for pipe in ("split", "staged", "mega", "refill"):
    os.environ["RT_PIPELINE"] = pipe
    for land in ("nomadplains", "testing"):
        for name, eul in (("reset", G.camera.INITIAL_ROTATION_EULER), ("down", G.camera.LOOKDOWN_ROTATION_EULER)):
            dev = G.DeviceFactory.construct(G.DeviceAPI.HIP, W, H, float_output=True, stats=True)
            ter = G.Terrain(dev, land); ter.create(); ter.reload()
            cam = G.Camera(W, H, euler=eul); ter.set_camera(cam); ter.set_time_of_day(0.3)
            ter.render_device(); dev.synchronize()
            img = dev.readback_float(); img8 = dev.readback(); st = dev.stats()
            ref = O.render(nz, O.make_frame(G.frame_constants(W, H, euler=eul), landscape=O.LANDSCAPES[land]))
            eq = (img.view(np.uint32) == ref['rgba32f'].view(np.uint32)).all(-1)
            print(pipe, land, name, 'bitexact', eq.mean(), 'u8', (img8 == ref['rgba8']).all(-1).mean(),
                  'steps gpu/oracle', st['primary_steps'], ref['stats']['primary_steps'], st['shadow_steps'], ref['stats']['shadow_steps'],
                  'noise', st['noise_calls'], ref['stats']['noise3d_calls'], flush=True)
            dev.destroy()
