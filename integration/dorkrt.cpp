// dorkrt -- the reference's CLI flow (src/main.cpp:132-202) with the reference's own parser
// and object model, rendering through librtgpu: Scene::loadFromXml builds the reference's
// DorkTracer::Scene exactly as its raytracer binary does; the adapter (dork_adapter.cpp)
// flattens it into an rtg_scene_desc; one rtg_render per camera replaces the 8-thread
// row-band block (main.cpp:164-185); the images are written with the reference's own
// stb writers (main.cpp:187-197).  Same argv and outputs as the reference:
//
//   dorkrt <scene.xml> [--devices N | --devices d0,d1,...]
//   dorkrt --compare <scene.xml>     adapter description == rtg_host_scene_load_xml's, field by field
//
// Built only where /root/reference exists (integration/Makefile); never copies its sources.
#define STB_IMAGE_WRITE_IMPLEMENTATION
#include "stb_image_write.h"
#define STB_IMAGE_IMPLEMENTATION
#define TINYEXR_IMPLEMENTATION

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "scene.h"
#include "tinyexr.h"
#include "dork_adapter.hpp"
#include "rtgpu.h"

namespace {

int die(const char* what) {
    std::fprintf(stderr, "dorkrt: %s: %s\n", what, rtg_last_error());
    return 1;
}

// ---- --compare: every array of the two descriptions, byte for byte (pointers cleared)
int mismatches = 0;

template <typename T>
void cmp_array(const char* name, const T* a, int64_t na, const T* b, int64_t nb, void (*clear)(T&) = nullptr) {
    if (na != nb) {
        std::printf("MISMATCH %s: count %lld vs %lld\n", name, (long long)na, (long long)nb);
        ++mismatches;
        return;
    }
    for (int64_t i = 0; i < na; ++i) {
        T x = a[i], y = b[i];
        if (clear) { clear(x); clear(y); }
        if (std::memcmp(&x, &y, sizeof(T))) {
            const unsigned char* p = reinterpret_cast<const unsigned char*>(&x);
            const unsigned char* q = reinterpret_cast<const unsigned char*>(&y);
            size_t k = 0;
            while (k < sizeof(T) && p[k] == q[k]) ++k;
            std::printf("MISMATCH %s[%lld]: first differing byte %zu of %zu\n", name, (long long)i, k, sizeof(T));
            ++mismatches;
            return;
        }
    }
    std::printf("equal %s (%lld)\n", name, (long long)na);
}

int compare(const char* xml) {
    DorkTracer::Scene scene;
    scene.loadFromXml(xml);
    rtg_dork::DescOwner D;
    std::string err;
    if (int rc = rtg_dork::desc_from_scene(scene, D, err)) {
        std::fprintf(stderr, "dorkrt: adapter: %s\n", err.c_str());
        return rc == RTG_ERR_UNSUPPORTED ? 3 : 1;
    }
    rtg_host_scene* hs = nullptr;
    if (rtg_host_scene_load_xml(xml, &hs)) return die("rtg_host_scene_load_xml");
    const rtg_scene_desc& a = D.desc;
    const rtg_scene_desc& b = *rtg_host_scene_desc(hs);
    if (std::memcmp(a.background, b.background, sizeof(a.background)) || a.shadow_epsilon != b.shadow_epsilon ||
        a.max_recursion_depth != b.max_recursion_depth || a.bg_texture != b.bg_texture ||
        std::memcmp(&a.ambient_light, &b.ambient_light, sizeof(rtg_float3))) {
        std::printf("MISMATCH scene header\n");
        ++mismatches;
    } else {
        std::printf("equal scene header\n");
    }
    cmp_array("cameras", a.cameras, a.num_cameras, b.cameras, b.num_cameras);
    cmp_array("materials", a.materials, a.num_materials, b.materials, b.num_materials);
    cmp_array("brdfs", a.brdfs, a.num_brdfs, b.brdfs, b.num_brdfs);
    cmp_array("point_lights", a.point_lights, a.num_point_lights, b.point_lights, b.num_point_lights);
    cmp_array("area_lights", a.area_lights, a.num_area_lights, b.area_lights, b.num_area_lights);
    cmp_array("dir_lights", a.dir_lights, a.num_dir_lights, b.dir_lights, b.num_dir_lights);
    cmp_array("spot_lights", a.spot_lights, a.num_spot_lights, b.spot_lights, b.num_spot_lights);
    cmp_array("env_lights", a.env_lights, a.num_env_lights, b.env_lights, b.num_env_lights);
    cmp_array("textures", a.textures, a.num_textures, b.textures, b.num_textures);
    cmp_array<rtg_image>("images", a.images, a.num_images, b.images, b.num_images,
                         [](rtg_image& im) { im.texels = nullptr; });
    for (int i = 0; i < a.num_images && i < b.num_images; ++i) {
        const int64_t n = (int64_t)a.images[i].width * a.images[i].height * a.images[i].channels;
        cmp_array("image texels", a.images[i].texels, n, b.images[i].texels, n);
    }
    cmp_array("objects", a.objects, a.num_objects, b.objects, b.num_objects);
    // surface_area: the reference leaves Mesh::surfaceArea uninitialised (mesh.cpp:7-13); both
    // sides use the sum of the face areas, in different orders -> compared to 1e-12 apart
    cmp_array<rtg_mesh>("meshes", a.meshes, a.num_meshes, b.meshes, b.num_meshes,
                        [](rtg_mesh& m) { m.surface_area = 0.0; });
    for (int i = 0; i < a.num_meshes && i < b.num_meshes; ++i)
        if (std::fabs(a.meshes[i].surface_area - b.meshes[i].surface_area) > 1e-12 * std::fabs(b.meshes[i].surface_area)) {
            std::printf("MISMATCH meshes[%d].surface_area %.17g vs %.17g\n", i, a.meshes[i].surface_area,
                        b.meshes[i].surface_area);
            ++mismatches;
        }
    cmp_array("faces", a.faces, a.num_faces, b.faces, b.num_faces);
    cmp_array("nodes", a.nodes, a.num_nodes, b.nodes, b.num_nodes);
    cmp_array("mesh_lights", a.mesh_lights, a.num_mesh_lights, b.mesh_lights, b.num_mesh_lights);
    rtg_host_scene_free(hs);
    std::printf("%s\n", mismatches ? "DIFFERENT" : "IDENTICAL");
    return mismatches ? 2 : 0;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc >= 3 && !std::strcmp(argv[1], "--compare")) return compare(argv[2]);
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s <scene.xml> [--devices N | d0,d1,...] | --compare <scene.xml>\n", argv[0]);
        return 2;
    }
    std::vector<int32_t> devices(1, 0);
    for (int i = 2; i + 1 < argc; ++i)
        if (!std::strcmp(argv[i], "--devices")) {
            std::string s = argv[i + 1];
            devices.clear();
            if (s.find(',') == std::string::npos) {
                for (int d = 0; d < std::atoi(s.c_str()); ++d) devices.push_back(d);
            } else {
                size_t p = 0;
                while (p <= s.size()) {
                    size_t q = s.find(',', p);
                    if (q == std::string::npos) q = s.size();
                    devices.push_back(std::atoi(s.substr(p, q - p).c_str()));
                    p = q + 1;
                }
            }
            if (devices.empty()) devices.assign(1, 0);
        }

    // main.cpp:135-137: the reference's parser builds its object model
    DorkTracer::Scene scene;
    scene.loadFromXml(argv[1]);
    auto start = std::chrono::steady_clock::now();

    // main.cpp:140 constructs a Raytracer (a copy of the scene); here the device replicas
    rtg_dork::DescOwner D;
    std::string err;
    if (rtg_dork::desc_from_scene(scene, D, err)) {
        std::fprintf(stderr, "dorkrt: %s\n", err.c_str());
        return 1;
    }
    rtg_scene* gpu = nullptr;
    if (rtg_scene_create_multi(&D.desc, devices.data(), (int32_t)devices.size(), &gpu)) return die("rtg_scene_create_multi");

    for (size_t i = 0; i < scene.cameras.size(); i++) {                 // main.cpp:142-197
        DorkTracer::Camera& cam = scene.cameras[i];
        const int width = cam.imageWidth, height = cam.imageHeight;
        const size_t n = (size_t)width * height * 3;
        void* image = nullptr;
        void* hdrImage = nullptr;
        if (rtg_host_alloc(n, &image)) return die("rtg_host_alloc");
        if (cam.hasTonemapper && rtg_host_alloc(n * sizeof(float), &hdrImage)) return die("rtg_host_alloc");
        if (cam.IsPathTracingEnabled()) std::printf("Path tracing is enabled for:%s\n", cam.imageName.c_str());
        std::printf("Resolution: %dx%d, Running on: %zu GPU(s).\n", width, height, devices.size());
        rtg_render_opts o;
        std::memset(&o, 0, sizeof(o));
        o.camera = (int32_t)i;
        o.sample_count = -1;
        o.seed = 0x5eed;
        // the 8 row-band threads -> one call; a tonemapped camera's LDR output is the
        // tonemapped image (main.cpp:187-192)
        if (rtg_render(gpu, &o, (float*)hdrImage, (uint8_t*)image)) return die("rtg_render");
        if (cam.hasTonemapper) stbi_write_hdr(cam.imageName.c_str(), width, height, 3, (const float*)hdrImage);
        size_t lastDot = cam.imageName.find_last_of(".");
        stbi_write_png((cam.imageName.substr(0, lastDot) + ".png").c_str(), width, height, 3, image, width * 3);
        rtg_host_free(image);
        if (hdrImage) rtg_host_free(hdrImage);
    }
    auto end = std::chrono::steady_clock::now();
    std::chrono::duration<double> elapsed_seconds = end - start;
    std::printf("Rendering took: %gs\n", elapsed_seconds.count());
    rtg_scene_destroy(gpu);
    return 0;
}
