// rtgpu -- drop-in for the reference CLI `raytracer <scene.xml>` (src/main.cpp:132-202).
// Same argv and outputs: for every camera, <ImageName stem>.png (LDR clamp) and, for a
// tonemapped camera, the raw float image via rtg_write_hdr.  The 8-thread row-band
// block (main.cpp:164-185) is replaced by one rtg_render call per camera.  The BVH is built
// on the GPU (RTG_LOAD_DEVICE_BVH; bit-identical to the reference's build); --host-bvh builds
// it on the CPU instead.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "rtgpu.h"

static int die(const char* what) {
    std::fprintf(stderr, "rtgpu: %s: %s\n", what, rtg_last_error());
    return 1;
}

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s <scene.xml> [--device N] [--host-bvh]\n", argv[0]);
        return 2;
    }
    int device = 0;
    uint32_t flags = RTG_LOAD_DEVICE_BVH;
    for (int i = 2; i < argc; ++i) {
        if (!std::strcmp(argv[i], "--device") && i + 1 < argc) device = std::atoi(argv[i + 1]);
        if (!std::strcmp(argv[i], "--host-bvh")) flags = 0;
    }

    rtg_host_scene* hs = nullptr;
    if (rtg_host_scene_load_xml_ex(argv[1], flags, &hs)) return die("loading scene");
    const rtg_scene_desc* desc = rtg_host_scene_desc(hs);
    auto start = std::chrono::steady_clock::now();
    rtg_scene* scene = nullptr;
    if (rtg_scene_create(desc, device, &scene)) return die("creating device scene");
    for (int c = 0; c < desc->num_cameras; ++c) {
        int32_t w, h, spp, tm;
        rtg_desc_camera_info(desc, c, &w, &h, &spp, &tm);
        std::printf("Resolution: %dx%d, Running on: HIP device %d.\n", w, h, device);
        std::vector<float> hdr((size_t)w * h * 3);
        std::vector<uint8_t> ldr((size_t)w * h * 3);
        rtg_render_opts o;
        std::memset(&o, 0, sizeof(o));
        o.camera = c;
        o.sample_count = -1;
        o.seed = 0x5eed;
        if (rtg_render(scene, &o, hdr.data(), ldr.data())) return die("rendering");
        std::string name = desc->cameras[c].image_name;
        if (tm) {
            if (rtg_write_hdr(name.c_str(), w, h, hdr.data())) return die("writing HDR");
        }
        size_t dot = name.find_last_of('.');
        std::string png = name.substr(0, dot) + ".png";
        if (rtg_write_png(png.c_str(), w, h, ldr.data())) return die("writing PNG");
    }
    auto end = std::chrono::steady_clock::now();
    std::printf("Rendering took: %gs\n", std::chrono::duration<double>(end - start).count());
    rtg_scene_destroy(scene);
    rtg_host_scene_free(hs);
    return 0;
}
