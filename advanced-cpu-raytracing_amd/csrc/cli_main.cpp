// rtgpu -- drop-in for the reference CLI `raytracer <scene.xml>` (src/main.cpp:132-202).
// Same argv and outputs: for every camera, <ImageName stem>.png (LDR clamp) and, for a
// tonemapped camera, the raw float image via rtg_write_hdr.  The 8-thread row-band
// block (main.cpp:164-185) is replaced by one rtg_render call per camera.  The BVH is built
// on the GPU (RTG_LOAD_DEVICE_BVH; bit-identical to the reference's build); --host-bvh builds
// it on the CPU instead.  --devices 0,1,... (or --devices N for the first N GPUs) deals the
// frame's 16-row bands to several GPUs of the node (rtg_scene_create_multi), each GPU copying
// its rows straight into the one page-locked host frame -- the reference's row-band threads
// (main.cpp:38-39,164-185) become GPUs; the image is bit-identical to a one-GPU render.
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
        std::fprintf(stderr, "usage: %s <scene.xml> [--device N | --devices N | --devices d0,d1,...] [--host-bvh]\n",
                     argv[0]);
        return 2;
    }
    std::vector<int32_t> devices(1, 0);
    uint32_t flags = RTG_LOAD_DEVICE_BVH;
    for (int i = 2; i < argc; ++i) {
        if (!std::strcmp(argv[i], "--device") && i + 1 < argc) devices.assign(1, std::atoi(argv[i + 1]));
        if (!std::strcmp(argv[i], "--devices") && i + 1 < argc) {
            std::string a = argv[i + 1];
            devices.clear();
            if (a.find(',') == std::string::npos) {
                for (int d = 0; d < std::atoi(a.c_str()); ++d) devices.push_back(d);
            } else {
                size_t p = 0;
                while (p <= a.size()) {
                    size_t q = a.find(',', p);
                    if (q == std::string::npos) q = a.size();
                    devices.push_back(std::atoi(a.substr(p, q - p).c_str()));
                    p = q + 1;
                }
            }
            if (devices.empty()) devices.assign(1, 0);
        }
        if (!std::strcmp(argv[i], "--host-bvh")) flags = 0;
    }

    rtg_host_scene* hs = nullptr;
    if (rtg_host_scene_load_xml_ex(argv[1], flags, &hs)) return die("loading scene");
    const rtg_scene_desc* desc = rtg_host_scene_desc(hs);
    auto start = std::chrono::steady_clock::now();
    rtg_scene* scene = nullptr;
    if (rtg_scene_create_multi(desc, devices.data(), (int32_t)devices.size(), &scene))
        return die("creating device scene");
    for (int c = 0; c < desc->num_cameras; ++c) {
        int32_t w, h, spp, tm;
        rtg_desc_camera_info(desc, c, &w, &h, &spp, &tm);
        std::printf("Resolution: %dx%d, Running on: %zu HIP device(s).\n", w, h, devices.size());
        // page-locked frame: every GPU's part is one DMA into it (main.cpp:146-152 news it)
        const size_t n = (size_t)w * h * 3;
        void* hdr = nullptr;
        void* ldr = nullptr;
        if (tm && rtg_host_alloc(n * sizeof(float), &hdr)) return die("allocating the HDR frame");
        if (rtg_host_alloc(n, &ldr)) return die("allocating the LDR frame");
        rtg_render_opts o;
        std::memset(&o, 0, sizeof(o));
        o.camera = c;
        o.sample_count = -1;
        o.seed = 0x5eed;
        if (rtg_render(scene, &o, (float*)hdr, (uint8_t*)ldr)) return die("rendering");
        std::string name = desc->cameras[c].image_name;
        if (tm) {
            if (rtg_write_hdr(name.c_str(), w, h, (const float*)hdr)) return die("writing HDR");
        }
        size_t dot = name.find_last_of('.');
        std::string png = name.substr(0, dot) + ".png";
        if (rtg_write_png(png.c_str(), w, h, (const uint8_t*)ldr)) return die("writing PNG");
        rtg_host_free(hdr);
        rtg_host_free(ldr);
    }
    auto end = std::chrono::steady_clock::now();
    std::printf("Rendering took: %gs\n", std::chrono::duration<double>(end - start).count());
    rtg_scene_destroy(scene);
    rtg_host_scene_free(hs);
    return 0;
}
