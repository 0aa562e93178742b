"""gpgpuraytrace_amd -- MI355X-native (gfx950 HIP) drop-in for MadrMan/gpgpuraytrace's
hot path: camerarays -> tracescreen -> traceRay -> getDensity -> noise3d, shading,
shadow ray and sky, behind the reference's ICompute/IDevice dispatch-and-readback
surface (C-ABI: include/frosttrace.h, library: gpgpuraytrace_amd/_build/librt_hip.so).
"""
from ._native import LIB_PATH, NativeError, lib  # noqa: F401
from .camera import Camera, frame_constants, sun_direction  # noqa: F401
from .engine import (Compute, Device, DeviceAPI, DeviceFactory, FrameRing, Noise, Recorder, RecorderFactory,  # noqa: F401
                     ShaderArray, ShaderVariable, Terrain, Texture, VariableManager, read_recording,
                     set_target_depths_host, vfs_add_path, vfs_clear)

__all__ = ["Camera", "Compute", "Device", "DeviceAPI", "DeviceFactory", "FrameRing", "Noise", "Recorder", "RecorderFactory", "read_recording", "VariableManager", "ShaderArray", "ShaderVariable",
           "Terrain", "Texture", "frame_constants", "sun_direction", "vfs_add_path", "vfs_clear", "lib", "LIB_PATH"]
