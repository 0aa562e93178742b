// hip_adapter.cpp -- see hip_adapter.h.
#include "hip_adapter.h"

#include "Common/Timer.h"

TextureHIP::TextureHIP(rt_device dev) { rt_texture_create(dev, &tex); }
TextureHIP::~TextureHIP() { rt_texture_destroy(tex); }

// Loading textures from disk is not on the terrain path (Terrain only builds perm2D
// from memory, Terrain.cpp:55-62); it fails like an unreadable file does.
bool TextureHIP::create(const std::string&) { return false; }

bool TextureHIP::create(TextureDimensions::T dimensions, TextureFormat::T format, int width, int height,
                        const void* data, TextureBinding::T binding, CPUAccess::T cpuFlags)
{
    return tex && rt_texture_init(tex, (int)dimensions, (int)format, width, height, data, (int)binding,
                                  (int)cpuFlags) == RT_OK;
}

ComputeHIP::ComputeHIP(rt_device dev) { rt_compute_create(dev, &cs); }
ComputeHIP::~ComputeHIP() { rt_compute_destroy(cs); }

bool ComputeHIP::create(const std::string& directory, const std::string& fileName, const std::string& main,
                        const ThreadSize& ts, const std::vector<MacroType>& macros)
{
    std::vector<const char*> names, values;
    for (const MacroType& m : macros) {
        names.push_back(m.first.c_str());
        values.push_back(m.second.c_str());
    }
    if (rt_compute_load(cs, directory.c_str(), fileName.c_str(), main.c_str(), ts.x, ts.y, ts.z, names.data(),
                        values.data(), (int)macros.size()) != RT_OK)
        return false; // the previous shader stays current (ComputeDirect3D.cpp:403-465)
    pending = ts;
    return true;
}

void ComputeHIP::run(unsigned int dispatchX, unsigned int dispatchY, unsigned int dispatchZ)
{
    rt_compute_run(cs, dispatchX, dispatchY, dispatchZ);
}

IShaderVariable* ComputeHIP::getVariable(const std::string& name)
{
    auto it = variables.find(name);
    if (it != variables.end()) return it->second.get();
    rt_variable v = rt_compute_get_variable(cs, name.c_str());
    if (!v) return nullptr;
    return (variables[name] = std::unique_ptr<ShaderVariableHIP>(new ShaderVariableHIP(name, v))).get();
}

IShaderArray* ComputeHIP::getArray(const std::string& name)
{
    auto it = arrays.find(name);
    if (it != arrays.end()) return it->second.get();
    rt_array a = rt_compute_get_array(cs, name.c_str());
    if (!a) return nullptr;
    return (arrays[name] = std::unique_ptr<ShaderArrayHIP>(new ShaderArrayHIP(name, a))).get();
}

// ComputeDirect3D.cpp:121,138-141: the D3D type mask makes getBuffer always nullptr.
IShaderBuffer* ComputeHIP::getBuffer(const std::string&) { return nullptr; }

bool ComputeHIP::swap()
{
    if (rt_compute_swap(cs) != 1) return false;
    // variables/arrays belong to the replaced shader (ComputeDirect3D.cpp:91-100)
    variables.clear();
    arrays.clear();
    threadSize = pending;
    return true;
}

void ComputeHIP::setTexture(int stage, ITexture* texture)
{
    TextureHIP* t = dynamic_cast<TextureHIP*>(texture);
    rt_compute_set_texture(cs, stage, t ? t->handle() : nullptr);
}

DeviceHIP::DeviceHIP(IWindow* window) : IDevice(kDeviceApiHip, window) { }
DeviceHIP::~DeviceHIP() { rt_device_destroy(dev); }

bool DeviceHIP::create()
{
    const WindowSettings& ws = getWindow()->getWindowSettings();
    return rt_device_create(ws.gpu < 0 ? 0 : ws.gpu, ws.width, ws.height, flags, &dev) == RT_OK;
}

void DeviceHIP::present()
{
    // the recorder's sample duration when not fixed speed (RecorderWinAPI.cpp:264-269)
    if (recorder) rt_recorder_set_frame_time(recorder->handle(), Timer::get()->getConstant());
    rt_device_present(dev);
}
void DeviceHIP::flush() { rt_device_flush(dev); }
ICompute* DeviceHIP::createCompute() { return new ComputeHIP(dev); }
ITexture* DeviceHIP::createTexture() { return new TextureHIP(dev); }

bool DeviceHIP::readback(void* dst, size_t rowPitch) const { return rt_device_readback(dev, dst, rowPitch) == RT_OK; }

bool RecorderHIP::create()
{
    DeviceHIP* d = dynamic_cast<DeviceHIP*>(device);
    if (!d || rt_recorder_create(d->handle(), frameRate, fixedSpeed ? 1 : 0, "output.rgb32", &rec) != RT_OK)
        return false;
    d->setRecorder(this);
    return true;
}

RecorderHIP::~RecorderHIP()
{
    if (DeviceHIP* d = dynamic_cast<DeviceHIP*>(device)) d->setRecorder(nullptr);
    rt_recorder_destroy(rec);
}
