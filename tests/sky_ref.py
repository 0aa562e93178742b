"""Float64 numpy restatement of the reference sky (TEST INFRASTRUCTURE, an independent checker).

Follows Media/common/shaders/sky.hlsl line by line in double precision with exact
transcendentals (numpy exp / power), and Media/common/shaders/noise.hlsl:139-179 (the live
`#if 1` noise3d) for the star field, on the perm2D / permGradients tables the caller passes.
It shares no code and no evaluation rule with oracle/rt_oracle.c (float32, fixed fma and
polynomial conventions), so agreement within a tolerance pins the oracle's sky arithmetic to the
HLSL's real-number meaning.
"""
import numpy as np

# sky.hlsl:1-16 (const static)
F_SAMPLES = 3.0
N_SAMPLES = 3
SCALE_DEPTH = np.float64(np.float32(0.19))
E_SPACE = 1.0
E_SUN = 12.0
KR = np.float64(np.float32(0.003))
KM = np.float64(np.float32(0.0025))
PI = np.float64(np.float32(3.14159265))
INNER = 200.0
OUTER = INNER * np.float64(np.float32(1.025))
WAVELENGTH = np.array([0.650, 0.570, 0.475], np.float32).astype(np.float64)
WAVELENGTH4 = WAVELENGTH ** 4
G = np.float64(np.float32(-0.99))
# sky.hlsl:74-80
INV_WAVELENGTH = 1.0 / WAVELENGTH4
KR_ESUN = E_SUN * KR
KM_ESUN = E_SUN * KM
KR_4PI = KR * 4.0 * PI
KM_4PI = KM * 4.0 * PI
F_SCALE = 1.0 / (OUTER - INNER)
SCALE_OVER_SCALE_DEPTH = F_SCALE / SCALE_DEPTH


def _sat(x):
    return np.clip(x, 0.0, 1.0)


def _normalize(v):
    return v / np.linalg.norm(v, axis=-1, keepdims=True)


def mod_ray_dir(d):
    """sky.hlsl:18-23"""
    d = np.array(d, np.float64, copy=True)
    d[..., 1] = _sat(d[..., 1])
    return _normalize(d)


def _scale(fcos):
    """sky.hlsl:39-43"""
    x = 1.0 - fcos
    return SCALE_DEPTH * np.exp(-0.00287 + x * (0.459 + x * (3.83 + x * (-6.80 + x * 5.25))))


def _mie_phase(fcos, fcos2, g, g2):
    """sky.hlsl:46-49"""
    return 1.5 * ((1.0 - g2) / (2.0 + g2)) * (1.0 + fcos2) / np.power(np.abs(1.0 + g2 - 2.0 * g * fcos), 1.5)


def rayleigh_mie(dirs, eye, sun):
    """getRayleighMieColor (sky.hlsl:83-137), applyPhase (:62-72) with the call's argument order
    (:131: applyPhase(mie, rayleigh, t) into the parameters (rayleigh, mie, camDir)).
    dirs (n, 3); returns (mie (n, 3), rayleigh (n, 3))."""
    org = np.asarray(dirs, np.float64).reshape(-1, 3)
    eye = np.asarray(eye, np.float64)
    sun = np.asarray(sun, np.float64)
    rd = mod_ray_dir(org)
    cam_h = max(INNER + eye[1] * 0.001, 0.0)
    dist_to_top = OUTER - cam_h
    far = dist_to_top + (1.0 - rd[:, 1]) * dist_to_top * 2.0
    start = np.array([eye[0] * 0.001, cam_h, eye[2] * 0.001])
    depth0 = np.exp(SCALE_OVER_SCALE_DEPTH * (INNER - cam_h))
    start_angle = rd @ _normalize(start)
    start_offset = depth0 * _scale(start_angle)
    sample_len = far / F_SAMPLES
    scaled_len = sample_len * F_SCALE
    sample_ray = rd * sample_len[:, None]
    sp = start[None, :] + sample_ray * 0.5
    front = np.zeros_like(rd)
    for _ in range(N_SAMPLES):
        h = np.linalg.norm(sp, axis=1)
        dep = np.exp(SCALE_OVER_SCALE_DEPTH * (INNER - h))
        light = (sp @ sun) / h
        camera = np.sum(rd * sp, axis=1) / h
        scatter = start_offset + dep * (_scale(light) - _scale(camera))
        att = np.exp(-scatter[:, None] * (INV_WAVELENGTH * KR_4PI + KM_4PI)[None, :])
        front += att * (dep * scaled_len)[:, None]
        sp = sp + sample_ray
    mie_var = front * (INV_WAVELENGTH * KR_ESUN)[None, :]
    ray_var = front * KM_ESUN
    t = -rd * far[:, None]
    # applyPhase(rayleigh := mie_var, mie := ray_var, camDir := t)
    fcos = (t @ sun) / np.linalg.norm(t, axis=1)
    fcos2 = fcos * fcos
    mie = _mie_phase(fcos, fcos2, G, G * G)[:, None] * ray_var
    rayleigh = (0.75 + 0.75 * fcos2)[:, None] * mie_var
    rayleigh = rayleigh * _sat((org[:, 1] * 0.5 + 0.5) * 4.0)[:, None]
    sy = _sat(sun[1])
    rayleigh = rayleigh + np.array([0.3, 0.4, 0.6]) * sy
    return mie, rayleigh


def noise3d(perm2d, grad, p):
    """noise.hlsl:139-179 (live block) in float64: perm2d (128*128*4) uint8, grad (128, 4)."""
    p = np.asarray(p, np.float64).reshape(-1, 3)
    P = np.floor(p)
    f = p - P
    u = f * f * f * (f * (f * 6.0 - 15.0) + 10.0)
    X, Y, Z = [(P[:, i].astype(np.int64) & 127) for i in range(3)]
    tex = perm2d.reshape(128, 128, 4)[Y, X].astype(np.int64)  # texel (x, y) at (x + y*128)*4
    g = np.asarray(grad, np.float64).reshape(128, 4)[:, :3]

    def gp(idx, x, y, z):
        gg = g[idx % 128]
        return gg[:, 0] * x + gg[:, 1] * y + gg[:, 2] * z

    x, y, z = f[:, 0], f[:, 1], f[:, 2]
    A, AB, B, BB = [tex[:, i] + Z for i in range(4)]  # Pu = texel + P.z (noise.hlsl:166)
    lerp = lambda a, b, t: a + t * (b - a)  # noqa: E731
    l0 = lerp(lerp(gp(A, x, y, z), gp(B, x - 1, y, z), u[:, 0]),
              lerp(gp(AB, x, y - 1, z), gp(BB, x - 1, y - 1, z), u[:, 0]), u[:, 1])
    l1 = lerp(lerp(gp(A + 1, x, y, z - 1), gp(B + 1, x - 1, y, z - 1), u[:, 0]),
              lerp(gp(AB + 1, x, y - 1, z - 1), gp(BB + 1, x - 1, y - 1, z - 1), u[:, 0]), u[:, 1])
    return lerp(l0, l1, u[:, 2])


def space_color(perm2d, grad, dirs, sun):
    """getSpaceColor (sky.hlsl:26-36): 0 below the horizon."""
    d = mod_ray_dir(np.asarray(dirs, np.float64).reshape(-1, 3))
    s = noise3d(perm2d, grad, d * 500.0)
    s = s - (noise3d(perm2d, grad, d * 150.2) * 0.5 + 0.13)
    s = s - (noise3d(perm2d, grad, d * 200.2) * 0.5 + 0.5)
    s = s * E_SPACE * _sat(-np.asarray(sun, np.float64)[1] * 2.7 - 0.5)
    return np.where(d[:, 1] <= 0.0, 0.0, s)
