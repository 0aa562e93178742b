// terrain_driver.cpp -- replays Graphics/Terrain.cpp's per-frame call sequence through the C++
// adapter (hip_adapter.{h,cpp}): every call goes through the reference's own interfaces
// (IDevice, ICompute, IShaderVariable, IShaderArray, ITexture; compiled against the reference
// headers), so this is what Terrain does once Factories/DeviceFactory.cpp constructs a DeviceHIP.
//
//   Terrain::create      (Terrain.cpp:55-89)   computes, noise tables, perm2D texture
//   Terrain::reload      (Terrain.cpp:91-103)  compute->create("shaders", "tracescreen.hlsl", ...)
//   calculateTileSizes   (Terrain.cpp:208-242)
//   Terrain::updateShaders (Terrain.cpp:138-206) swap -> getVariable / getArray -> write, setTexture
//   Terrain::render      (Terrain.cpp:105-136) run(2,2,1) -> CameraResults map/unmap ->
//                        setTargetDepths -> CellDistance write -> per tile ThreadOffset write +
//                        run + IDevice::flush; then IDevice::present (Raytracer.cpp:191)
//
// The frame constants come from a file the test writes (the engine's Camera output as the
// cbuffer bytes Terrain writes), so the driver needs no camera maths.
//   usage: terrain_driver <consts.bin> <out.bin> <landscape> <aa> <max_steps> <ao> <mode: ref|device|deferred>
//   consts.bin: int32 W, H; float ViewInverse[16] (cbuffer bytes), Eye[4], Projection[16]
//               (cbuffer bytes), SunDirection[3]
//   out.bin:    W*H*4 bytes RGBA8 (IDevice readback), then 1024 float4 CameraResults
// Test infrastructure for tests/test_gpu_parity.py::test_cpp_adapter_terrain_sequence; built by
// integration/Makefile (needs the reference headers, so it is built here and shipped prebuilt).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "Common/Timer.h"
// One translation unit with the adapter: the reference's Common.h defines isnull() in the header
// without `inline` off Windows (its `finline` macro is empty there), so two TUs that include the
// reference headers cannot be linked together.
#include "hip_adapter.cpp"

namespace {

const int kCameraViewRes = 32;   // Gameplay/Flyby.h:6
const int kCameraThreadRes = 16; // Gameplay/Flyby.h:7

class DriverWindow : public IWindow
{
public:
    explicit DriverWindow(const WindowSettings& ws) : IWindow(WindowAPI::X11, ws) { }
    bool create() override { return true; }
    void show() override { }
    bool update() override { return true; }
    IInput* getInput() override { return nullptr; }
};

// the engine's frame timer (Common/Timer.cpp); a fixed 40 ms step here
class FixedTimer : public Timer
{
public:
    float getTime() override { return 0.0f; }
    float getConstant() override { return 0.04f; }
    void update() override { }
};

struct Consts {
    int w = 0, h = 0;
    float view_inverse[16], eye[4], projection[16], sun[3];
};

bool read_consts(const char* path, Consts& c)
{
    FILE* f = std::fopen(path, "rb");
    if (!f) return false;
    bool ok = std::fread(&c.w, 4, 1, f) == 1 && std::fread(&c.h, 4, 1, f) == 1 &&
              std::fread(c.view_inverse, 4, 16, f) == 16 && std::fread(c.eye, 4, 4, f) == 4 &&
              std::fread(c.projection, 4, 16, f) == 16 && std::fread(c.sun, 4, 3, f) == 3;
    std::fclose(f);
    return ok;
}

// Terrain.cpp:208-242
struct Tiles {
    int tilesX, tilesY, threadX, threadY, dispatchX, dispatchY;
};
Tiles calculate_tile_sizes(int resx, int resy, bool recording)
{
    const int divisor = recording ? 4 : 1;
    const int tpx = 1024 / divisor, tpy = 512 / divisor;
    Tiles t;
    t.tilesX = (int)std::ceil(resx / (float)tpx);
    t.tilesY = (int)std::ceil(resy / (float)tpy);
    const int tileX = resx / t.tilesX, tileY = resy / t.tilesY;
    t.threadX = t.threadY = 16;
    while (tileX % t.threadX) ++t.threadX;
    while (tileY % t.threadY) ++t.threadY;
    t.dispatchX = tileX / t.threadX;
    t.dispatchY = tileY / t.threadY;
    return t;
}

void write_var(ICompute* cs, const char* name, const void* data)
{
    if (IShaderVariable* v = cs->getVariable(name)) v->write(const_cast<void*>(data));
}

} // namespace

Timer* Timer::get()
{
    static FixedTimer timer;
    return &timer;
}

int main(int argc, char** argv)
{
    if (argc != 8) {
        std::fprintf(stderr, "usage: %s consts.bin out.bin landscape aa max_steps ao ref|device|deferred\n", argv[0]);
        return 2;
    }
    Consts k;
    if (!read_consts(argv[1], k)) {
        std::fprintf(stderr, "cannot read %s\n", argv[1]);
        return 2;
    }
    const std::string landscape = argv[3], mode = argv[7];
    const int aa = std::atoi(argv[4]), maxSteps = std::atoi(argv[5]), ao = std::atoi(argv[6]);

    rt_vfs_add_path(("Media/" + landscape).c_str()); // Terrain.cpp:23
    WindowSettings ws = {k.w, k.h, false, 0};
    DriverWindow window(ws);
    DeviceHIP device(&window);
    IDevice* dev = &device;
    if (mode == "deferred") device.setFlags(RT_DEVICE_DEFERRED); // (the frame loop with deferred submission)
    if (!dev->create()) {
        std::fprintf(stderr, "device: %s\n", rt_last_error());
        return 1;
    }

    // Terrain::create
    ICompute* compute = dev->createCompute();
    ICompute* cameraCompute = dev->createCompute();
    std::vector<unsigned char> perm2d(128 * 128 * 4);
    std::vector<float> perm1d(128 * 4);
    rt_noise_generate(300, 0, perm2d.data(), perm1d.data()); // Noise::generate(false), MSVC CRT rand
    ITexture* texNoise2D = dev->createTexture();
    if (!texNoise2D->create(TextureDimensions::Texture2D, TextureFormat::R8G8B8A8_UINT, 128, 128, perm2d.data(),
                            TextureBinding::Texture, CPUAccess::None)) {
        std::fprintf(stderr, "texture: %s\n", rt_last_error());
        return 1;
    }

    // Terrain::reload (the build extensions ride on their own macros)
    const Tiles t = calculate_tile_sizes(k.w, k.h, false);
    std::vector<MacroType> macros;
    if (aa != 1) macros.push_back(MacroType("AA_SAMPLES", std::to_string(aa)));
    if (maxSteps) macros.push_back(MacroType("RT_MAX_STEPS", std::to_string(maxSteps)));
    std::vector<MacroType> screenMacros = macros;
    if (ao) screenMacros.push_back(MacroType("RT_AO_SAMPLES", std::to_string(ao)));
    const ThreadSize screenThreads = {t.threadX, t.threadY, 1};
    const ThreadSize cameraThreads = {kCameraThreadRes, kCameraThreadRes, 1};
    if (!compute->create("shaders", "tracescreen.hlsl", "CSMain", screenThreads, screenMacros) ||
        !cameraCompute->create("shaders", "camerarays.hlsl", "CSMain", cameraThreads, macros)) {
        std::fprintf(stderr, "shader: %s\n", rt_last_error());
        return 1;
    }

    // Terrain::updateShaders
    const float screen[2] = {(float)k.w, (float)k.h};
    IShaderVariable *varView = nullptr, *varEye = nullptr, *varSun = nullptr, *varThreadOffset = nullptr;
    IShaderArray *varCellDistance = nullptr, *varCamResults = nullptr;
    if (compute->swap()) {
        varView = compute->getVariable("ViewInverse");
        varEye = compute->getVariable("Eye");
        varSun = compute->getVariable("SunDirection");
        varThreadOffset = compute->getVariable("ThreadOffset");
        varCellDistance = compute->getArray("CellDistance");
        if (varCellDistance) varCellDistance->create(kCameraViewRes * kCameraViewRes);
        write_var(compute, "Projection", k.projection);
        write_var(compute, "ScreenSize", screen);
        write_var(compute, "permGradients", perm1d.data());
        compute->setTexture(0, texNoise2D);
    }
    IShaderVariable *varCamView = nullptr, *varCamEye = nullptr;
    if (cameraCompute->swap()) {
        varCamView = cameraCompute->getVariable("ViewInverse");
        varCamEye = cameraCompute->getVariable("Eye");
        varCamResults = cameraCompute->getArray("CameraResults");
        if (varCamResults) varCamResults->create(kCameraViewRes * kCameraViewRes);
        write_var(cameraCompute, "Projection", k.projection);
        write_var(cameraCompute, "ScreenSize", screen);
        write_var(cameraCompute, "permGradients", perm1d.data());
        cameraCompute->setTexture(0, texNoise2D);
    }
    // Terrain::updateTerrain / setTimeOfDay (Terrain.cpp:285-311), before the first dispatch
    for (IShaderVariable* v : {varView, varCamView})
        if (v) v->write(k.view_inverse);
    for (IShaderVariable* v : {varEye, varCamEye})
        if (v) v->write(k.eye);
    if (varSun) varSun->write(k.sun);

    std::vector<float> cameraView(kCameraViewRes * kCameraViewRes * 4, 0.0f);
    if (mode == "device" || mode == "deferred") {
        // the one-call device path: prepass, device setTargetDepths, trace.  Deferred:
        // three frames of the Raytracer loop (render, present), each launched by the next render, the last by the
        // CameraResults map
        for (int i = 0; i < (mode == "deferred" ? 3 : 1); ++i) {
            if (rt_terrain_render(static_cast<ComputeHIP*>(cameraCompute)->handle(),
                                  static_cast<ComputeHIP*>(compute)->handle(), 0, 1) != RT_OK) {
                std::fprintf(stderr, "render: %s\n", rt_last_error());
                return 1;
            }
            if (mode == "deferred" && i < 2) dev->present();
        }
        void* cr = varCamResults ? varCamResults->map() : nullptr;
        if (cr) {
            std::memcpy(cameraView.data(), cr, cameraView.size() * sizeof(float));
            varCamResults->unmap();
        }
    } else {
        // Terrain::render
        const unsigned int n = (unsigned int)std::ceil(kCameraViewRes / (float)kCameraThreadRes);
        cameraCompute->run(n, n, 1);
        if (varCamResults) { // Terrain::getCameraResults (Terrain.cpp:441-452)
            void* fd = varCamResults->map();
            if (!fd) {
                std::fprintf(stderr, "map: %s\n", rt_last_error());
                return 1;
            }
            std::memcpy(cameraView.data(), fd, cameraView.size() * sizeof(float));
            varCamResults->unmap();
            std::vector<float> cells(kCameraViewRes * kCameraViewRes * 2);
            rt_terrain_set_target_depths(cameraView.data(), cells.data()); // Terrain::setTargetDepths
            if (varCellDistance) varCellDistance->write(cells.data());
        }
        if (varThreadOffset) {
            for (int x = 0; x < t.tilesX; ++x) {
                for (int y = 0; y < t.tilesY; ++y) {
                    const unsigned int off[2] = {(unsigned int)(x * t.dispatchX * t.threadX),
                                                 (unsigned int)(y * t.dispatchY * t.threadY)};
                    varThreadOffset->write(const_cast<unsigned int*>(off));
                    compute->run(t.dispatchX, t.dispatchY, 1);
                    dev->flush();
                }
            }
        } else {
            compute->run(t.dispatchX * t.tilesX, t.dispatchY * t.tilesY, 1);
        }
    }
    dev->present(); // Raytracer.cpp:191
    std::vector<unsigned char> rgba((size_t)k.w * k.h * 4);
    if (!device.readback(rgba.data(), (size_t)k.w * 4)) {
        std::fprintf(stderr, "readback: %s\n", rt_last_error());
        return 1;
    }
    FILE* f = std::fopen(argv[2], "wb");
    if (!f) return 1;
    std::fwrite(rgba.data(), 1, rgba.size(), f);
    std::fwrite(cameraView.data(), sizeof(float), cameraView.size(), f);
    std::fclose(f);
    delete compute; // Terrain owns its computes and texture (Terrain.cpp:55-62)
    delete cameraCompute;
    delete texNoise2D;
    return 0;
}
