// hip_adapter.h -- the reference engine's device interfaces implemented over the
// frosttrace C-ABI (include/frosttrace.h).  Drop-in for Adapters/DeviceDirect3D +
// ComputeDirect3D + ShaderVariableDirect3D + TextureDirect3D: Terrain, Raytracer and
// Flyby keep calling IDevice / ICompute / IShaderVariable / IShaderArray / ITexture.
//
// Compiled against the reference headers (-I gpuraytrace); see INTEGRATION.md.
#pragma once

#include <map>
#include <memory>
#include <string>
#include <vector>

#include "Factories/ICompute.h"
#include "Factories/IDevice.h"
#include "Factories/IRecorder.h"
#include "Factories/ITexture.h"
#include "frosttrace.h"

// DeviceAPI::HIP once Factories/IDevice.h gains it.
const DeviceAPI::T kDeviceApiHip = static_cast<DeviceAPI::T>(3);

// ShaderVariableDirect3D.cpp:59-90 / 195-202: write copies the reflected size into a
// shadow uploaded lazily on the next run.
class ShaderVariableHIP : public IShaderVariable
{
public:
    ShaderVariableHIP(const std::string& name, rt_variable v) : IShaderVariable(name, nullptr), v(v)
    { setWritable(true); }
    void write(void* data) override { rt_variable_write(v, data); }

private:
    rt_variable v;
};

// UAVBufferD3D (ShaderVariableDirect3D.cpp:92-193) and StructuredBufferD3D (:204-281).
class ShaderArrayHIP : public IShaderArray
{
public:
    ShaderArrayHIP(const std::string& name, rt_array a) : IShaderArray(name), a(a) { setWritable(true); }
    bool create(unsigned int elements) override { return rt_array_create(a, elements) == RT_OK; }
    void* map() override { return rt_array_map(a); }
    void unmap() override { rt_array_unmap(a); }
    void write(void* data) override { rt_array_write(a, data); }

private:
    rt_array a;
};

// TextureDirect3D.cpp:40-164
class TextureHIP : public ITexture
{
public:
    explicit TextureHIP(rt_device dev);
    ~TextureHIP() override;
    bool create(const std::string& path) override;
    bool create(TextureDimensions::T dimensions, TextureFormat::T format, int width, int height, const void* data,
                TextureBinding::T binding, CPUAccess::T cpuFlags) override;
    rt_texture handle() const { return tex; }

private:
    rt_texture tex = nullptr;
};

// ComputeDirect3D.cpp:403-614
class ComputeHIP : public ICompute
{
public:
    explicit ComputeHIP(rt_device dev);
    ~ComputeHIP() override;
    bool create(const std::string& directory, const std::string& fileName, const std::string& main,
                const ThreadSize& ts, const std::vector<MacroType>& macros) override;
    void run(unsigned int dispatchX, unsigned int dispatchY, unsigned int dispatchZ) override;
    IShaderVariable* getVariable(const std::string& name) override;
    IShaderArray* getArray(const std::string& name) override;
    IShaderBuffer* getBuffer(const std::string& name) override;
    bool swap() override;
    void setTexture(int stage, ITexture* texture) override;
    rt_compute handle() const { return cs; }

private:
    rt_compute cs = nullptr;
    ThreadSize pending{};
    std::map<std::string, std::unique_ptr<ShaderVariableHIP>> variables;
    std::map<std::string, std::unique_ptr<ShaderArrayHIP>> arrays;
};

// DeviceDirect3D.cpp:77-267.  present() ends the frame; the linear RGBA8 framebuffer
// stays in HBM and readback() copies it out (recorder / window blit).
class DeviceHIP : public IDevice
{
public:
    explicit DeviceHIP(IWindow* window);
    ~DeviceHIP() override;
    bool create() override;
    void present() override;
    void flush() override;
    ICompute* createCompute() override;
    ITexture* createTexture() override;
    bool readback(void* dst, size_t rowPitch) const;
    rt_device handle() const { return dev; }
    void setRecorder(class RecorderHIP* r) { recorder = r; } // DeviceDirect3D::setRecorder (:229-232)
    // (adapter extension, before create) rt_device_create's flags, e.g. RT_DEVICE_DEFERRED (ABI 9): the reference's
    // IDevice::create takes none
    void setFlags(unsigned f) { flags = f; }

private:
    rt_device dev = nullptr;
    unsigned flags = 0;
    class RecorderHIP* recorder = nullptr;
};

// RecorderWinAPI (Adapters/RecorderWinAPI.cpp) over rt_recorder_*: RecorderFactory::construct
// makes one for a DeviceHIP; it attaches to the device, whose present() then writes every
// frame while recording (DeviceDirect3D.cpp:242-256), swizzled to RGB32 on the GPU.  The sink
// is a raw-video file (+ time-stamp index) instead of Media Foundation's output.wmv.
class RecorderHIP : public IRecorder
{
public:
    RecorderHIP(IDevice* device, int frameRate, bool fixedSpeed) : device(device), frameRate(frameRate),
        fixedSpeed(fixedSpeed) { }
    ~RecorderHIP() override;
    bool create() override;
    void start() override { IRecorder::start(); rt_recorder_start(rec); }
    void stop() override { IRecorder::stop(); rt_recorder_stop(rec); }
    void write(void* frame, int stride) override { rt_recorder_write(rec, frame, stride); }
    rt_recorder handle() const { return rec; }

private:
    IDevice* device;
    int frameRate;
    bool fixedSpeed;
    rt_recorder rec = nullptr;
};
