import sys, time, os
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests')
import numpy as np
import gpgpuraytrace_amd as G
import oracle_lib as O
W, H = 64, 48
for name, eul in (("reset", G.camera.INITIAL_ROTATION_EULER), ("down", G.camera.LOOKDOWN_ROTATION_EULER)):
    dev = G.DeviceFactory.construct(G.DeviceAPI.HIP, W, H, float_output=True, stats=True)
    assert dev is not None, G.lib().rt_last_error()
    ter = G.Terrain(dev, "nomadplains"); ter.create(); ter.reload()
    cam = G.Camera(W, H, euler=eul); ter.set_camera(cam); ter.set_time_of_day(0.3)
    t = time.time(); ter.render_device(); dev.synchronize(); print(name, 'render_device %.3fs' % (time.time() - t))
    img = dev.readback_float(); img8 = dev.readback(); st = dev.stats()
    consts = G.frame_constants(W, H, euler=eul)
    ref = O.render(O.noise_tables(), O.make_frame(consts))
    d = np.abs(img - ref['rgba32f']); eq = (img.view(np.uint32) == ref['rgba32f'].view(np.uint32)).all(-1)
    print(name, 'bitexact px frac', eq.mean(), 'max abs', d.max(), 'u8 eq', (img8 == ref['rgba8']).all(-1).mean())
    print(name, 'gpu stats', st, 'oracle', ref['stats'])
    ter.render(); dev.synchronize()
    img2 = dev.readback_float()
    print(name, 'compat path bitexact frac', (img2.view(np.uint32) == ref['rgba32f'].view(np.uint32)).all(-1).mean())
