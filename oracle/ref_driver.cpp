// ORACLE -- test infrastructure only.  Driver linked against the reference's own
// sources (compiled from /root/reference/src by oracle/Makefile into oracle/_ref/;
// nothing of the reference is copied into this repository).
//
//   refdriver dump  <scene.xml> <out.bin> [camera]
//       Single-threaded loop calling Raytracer::RenderPixel(x, y, cam) for every pixel
//       of one camera (raytracer.hpp:19), i.e. the spp==1 path of renderThreadMain
//       (main.cpp:102-105).  Writes "RTGF" int32 w, int32 h, then w*h*3 float32 RGB,
//       row-major 3*(x+y*w) (main.cpp:109).  Deterministic scenes only (the reference's
//       random streams are seeded from rand() and raced by its threads).
//   refdriver dumpavg <scene.xml> <out.bin> <n> [camera]
//       Stochastic scenes (path tracing, area / environment lights): n RenderPixel calls per
//       pixel, single-threaded.  Writes "RTGV" int32 w, h, n, then the per-pixel mean and
//       the variance of that mean (w*h*3 float32 each) -- the statistical golden.
//   refdriver bench <scene.xml> <threads> <reps> [camera] [png] [row_begin row_end]
//       Times the reference's row-band render exactly as main.cpp:164-185 partitions it
//       (rows [t*(H/T), (t+1)*(H/T)) per thread; spawn -> join), each pixel as
//       renderThreadMain does it (main.cpp:42-121: one RenderPixel, or for spp > 1 the
//       stratified jitter from the thread's mt19937, spp RenderPixel calls and the Gaussian2D
//       weighting of gaussian.h), and the reference-equivalent span main.cpp:138-199
//       (Raytracer copy + render + PNG encode); prints one JSON line with the per-rep seconds
//       of both.  With row_begin / row_end only those rows are rendered (a bounded sample of a
//       long frame), dealt to the threads the same way.
//   refdriver imgdump <image file> <out.bin>
//       The reference's own image classes as parser.cpp:103-110 picks them: HDRImage (tinyexr
//       LoadEXR) for a ".exr" name, else LDRImage (stbi_load).  Writes "RTGI" int32 w, h,
//       channels, is_hdr, then w*h*channels float32 (the texel values GetSample reads).
//   refdriver tonemap <in.bin> <key> <burn%> <saturation> <gamma> <out.bin>
//       The reference's own Tonemapper::Tonemap (tonemapper.h:28-60) on an "RTGF" float
//       image (as dump writes); writes "RTGL" int32 w, int32 h, w*h*3 uint8 (the LDR
//       image main.cpp:187-195 saves for a tonemapped camera).
#define STB_IMAGE_WRITE_IMPLEMENTATION
#include "stb_image_write.h"
#define STB_IMAGE_IMPLEMENTATION
#define TINYEXR_IMPLEMENTATION

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <algorithm>
#include <vector>

#include <random>

#include "raytracer.hpp"
#undef STB_IMAGE_IMPLEMENTATION          // emitted once above (raytracer.hpp -> image.h)
#include "LDRImage.h"
#include "gaussian.h"

using namespace DorkTracer;

static int imgdump(const char* file, const char* out) {
    std::string name(file);
    int w = 0, h = 0, c = 0, hdr = 0;
    std::vector<float> t;
    if (name.find(".exr") != std::string::npos) {
        HDRImage im(name, 0);
        w = im.width; h = im.height; c = 3; hdr = 1;
        t.assign(im.src.begin(), im.src.end());
    } else {
        struct Peek : LDRImage {               // the loaded bytes (protected members)
            using LDRImage::LDRImage;
            const unsigned char* bytes() const { return image; }
            int nch() const { return channels; }
        } im(name, 0);
        if (!im.bytes()) return 1;
        w = im.width; h = im.height; c = im.nch();
        t.assign(im.bytes(), im.bytes() + (size_t)w * h * c);
    }
    FILE* f = std::fopen(out, "wb");
    if (!f) { std::perror(out); return 1; }
    int32_t hd[4] = {w, h, c, hdr};
    std::fwrite("RTGI", 1, 4, f);
    std::fwrite(hd, 4, 4, f);
    std::fwrite(t.data(), 4, t.size(), f);
    std::fclose(f);
    return 0;
}

static int dump(const char* xml, const char* out, int ci) {
    Scene scene;
    scene.loadFromXml(xml);
    Raytracer renderer(scene);
    if (ci < 0 || ci >= (int)scene.cameras.size()) { std::fprintf(stderr, "bad camera\n"); return 2; }
    Camera& cam = scene.cameras[ci];
    if (cam.IsPathTracingEnabled()) renderer.EnablePathTracing(cam.GetRendererParams());
    renderer.activeCamera = &cam;
    const int w = cam.imageWidth, h = cam.imageHeight;
    std::vector<float> img((size_t)w * h * 3);
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            Vec3f c = renderer.RenderPixel(x, y, cam);
            size_t i = 3 * ((size_t)x + (size_t)y * w);
            img[i] = c.x; img[i + 1] = c.y; img[i + 2] = c.z;
        }
    FILE* f = std::fopen(out, "wb");
    if (!f) { std::perror(out); return 1; }
    int32_t hdr[2] = {w, h};
    std::fwrite("RTGF", 1, 4, f);
    std::fwrite(hdr, sizeof(int32_t), 2, f);
    std::fwrite(img.data(), sizeof(float), img.size(), f);
    std::fclose(f);
    return 0;
}

static int dumpavg(const char* xml, const char* out, int n, int ci) {
    Scene scene;
    scene.loadFromXml(xml);
    Raytracer renderer(scene);
    if (ci < 0 || ci >= (int)scene.cameras.size() || n < 2) { std::fprintf(stderr, "bad camera / n\n"); return 2; }
    Camera& cam = scene.cameras[ci];
    if (cam.IsPathTracingEnabled()) renderer.EnablePathTracing(cam.GetRendererParams());
    renderer.activeCamera = &cam;
    const int w = cam.imageWidth, h = cam.imageHeight;
    std::vector<float> mean((size_t)w * h * 3), var((size_t)w * h * 3);
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            double s[3] = {0, 0, 0}, q[3] = {0, 0, 0};
            for (int k = 0; k < n; ++k) {
                Vec3f c = renderer.RenderPixel(x, y, cam);
                const double v[3] = {c.x, c.y, c.z};
                for (int j = 0; j < 3; ++j) { s[j] += v[j]; q[j] += v[j] * v[j]; }
            }
            size_t i = 3 * ((size_t)x + (size_t)y * w);
            for (int j = 0; j < 3; ++j) {
                const double m = s[j] / n;
                mean[i + j] = (float)m;
                var[i + j] = (float)(std::max(0.0, q[j] / n - m * m) / (n - 1));
            }
        }
    FILE* f = std::fopen(out, "wb");
    if (!f) { std::perror(out); return 1; }
    int32_t hdr[3] = {w, h, n};
    std::fwrite("RTGV", 1, 4, f);
    std::fwrite(hdr, sizeof(int32_t), 3, f);
    std::fwrite(mean.data(), sizeof(float), mean.size(), f);
    std::fwrite(var.data(), sizeof(float), var.size(), f);
    std::fclose(f);
    return 0;
}

// Per rep two clocks: "seconds" = spawn -> join of the row-band threads (render only,
// main.cpp:164-185); "span_seconds" = the reference's own "Rendering took" span
// main.cpp:138 -> 199 for one camera: Raytracer copy-construction (main.cpp:140), the
// LDR frame buffer, the threaded render with the clamp of main.cpp:118-124, and the PNG
// encode of main.cpp:197 (written to png_out, "" = /dev/null-like temp name).
// One pixel as renderThreadMain computes it (main.cpp:57-101), the thread's generator and
// sample vector passed in.
static Vec3f bench_pixel(Raytracer& renderer, Camera& cam, int x, int y, std::mt19937& gen,
                         std::uniform_real_distribution<>& u01, std::vector<Vec2f>& samples, Gaussian2D& g) {
    const int spp = cam.samplesPerPixel;
    if (spp <= 1) return renderer.RenderPixel(x, y, cam);
    const int n = (int)std::sqrt(spp);
    int i = 0;
    for (int r = 0; r < n; ++r)
        for (int c = 0; c < n; ++c) {
            const float p1 = u01(gen), p2 = u01(gen);
            samples[i].x = (c + p1) / n;
            samples[i].y = (r + p2) / n;
            ++i;
        }
    Vec3f col{0.0f, 0.0f, 0.0f};
    float wsum = 0.0f;
    for (i = 0; i < spp; ++i) {
        // (RenderPixel takes int coordinates: the jitter only moves the Gaussian weight)
        const Vec3f v = renderer.RenderPixel(samples[i].x + x, samples[i].y + y, cam);
        const float gw = g.GetWeight(samples[i].x - 0.5f, samples[i].y - 0.5f);
        col.x += v.x * gw;
        col.y += v.y * gw;
        col.z += v.z * gw;
        wsum += gw;
    }
    col.x = col.x / wsum;
    col.y = col.y / wsum;
    col.z = col.z / wsum;
    return col;
}

static int bench(const char* xml, int threads, int reps, int ci, const char* png_out, int rb, int re) {
    Scene scene;
    scene.loadFromXml(xml);
    Camera& cam = scene.cameras[ci];
    const int w = cam.imageWidth, h = cam.imageHeight;
    if (re <= 0 || re > h) re = h;
    if (rb < 0 || rb >= re) rb = 0;
    const int band = re - rb;
    std::vector<float> img((size_t)w * h * 3);
    std::vector<double> render_s, span_s;
    for (int r = 0; r < reps; ++r) {
        auto s0 = std::chrono::steady_clock::now();
        Raytracer renderer(scene);
        renderer.activeCamera = &cam;
        std::vector<unsigned char> ldr((size_t)w * h * 3);
        auto t0 = std::chrono::steady_clock::now();
        std::vector<std::thread> th;
        for (int t = 0; t < threads; ++t) {
            th.emplace_back([&, t]() {
                int y0 = rb + t * (band / threads), y1 = y0 + band / threads;
                std::mt19937 gen(rand());
                std::uniform_real_distribution<> u01(0.0f, 1.0f);
                std::vector<Vec2f> samples(std::max(1, cam.samplesPerPixel));
                Gaussian2D g(1.0f / 6.0f);
                for (int y = y0; y < y1; ++y)
                    for (int x = 0; x < w; ++x) {
                        Vec3f c = bench_pixel(renderer, cam, x, y, gen, u01, samples, g);
                        size_t i = 3 * ((size_t)x + (size_t)y * w);
                        img[i] = c.x; img[i + 1] = c.y; img[i + 2] = c.z;
                        Vec3i q = clamp(c);
                        ldr[i] = q.x; ldr[i + 1] = q.y; ldr[i + 2] = q.z;
                    }
            });
        }
        for (auto& t : th) t.join();
        auto t1 = std::chrono::steady_clock::now();
        stbi_write_png(png_out, w, h, 3, ldr.data(), w * 3);
        auto s1 = std::chrono::steady_clock::now();
        render_s.push_back(std::chrono::duration<double>(t1 - t0).count());
        span_s.push_back(std::chrono::duration<double>(s1 - s0).count());
    }
    double checksum = 0;
    for (float v : img) checksum += v;
    std::printf("{\"threads\": %d, \"width\": %d, \"height\": %d, \"spp\": %d, \"rows\": [%d, %d], \"seconds\": [",
                threads, w, h, cam.samplesPerPixel, rb, rb + (band / threads) * threads);
    for (size_t r = 0; r < render_s.size(); ++r) std::printf("%s%.6f", r ? ", " : "", render_s[r]);
    std::printf("], \"span_seconds\": [");
    for (size_t r = 0; r < span_s.size(); ++r) std::printf("%s%.6f", r ? ", " : "", span_s[r]);
    std::printf("], \"checksum\": %.6f}\n", checksum);
    return 0;
}

static int tonemap(const char* in, float key, float burn, float sat, float gamma, const char* out) {
    FILE* f = std::fopen(in, "rb");
    if (!f) { std::perror(in); return 1; }
    char magic[4];
    int32_t wh[2];
    if (std::fread(magic, 1, 4, f) != 4 || std::memcmp(magic, "RTGF", 4) || std::fread(wh, 4, 2, f) != 2) return 1;
    std::vector<float> hdr((size_t)wh[0] * wh[1] * 3);
    if (std::fread(hdr.data(), 4, hdr.size(), f) != hdr.size()) return 1;
    std::fclose(f);
    std::vector<unsigned char> ldr(hdr.size());
    Tonemapper tm("Photographic", key, burn, sat, gamma);
    tm.Tonemap(wh[0], wh[1], hdr.data(), ldr.data());
    f = std::fopen(out, "wb");
    if (!f) { std::perror(out); return 1; }
    std::fwrite("RTGL", 1, 4, f);
    std::fwrite(wh, 4, 2, f);
    std::fwrite(ldr.data(), 1, ldr.size(), f);
    std::fclose(f);
    return 0;
}

int main(int argc, char** argv) {
    if (argc >= 8 && !std::strcmp(argv[1], "tonemap"))
        return tonemap(argv[2], std::atof(argv[3]), std::atof(argv[4]), std::atof(argv[5]), std::atof(argv[6]), argv[7]);
    if (argc >= 4 && !std::strcmp(argv[1], "dump")) return dump(argv[2], argv[3], argc > 4 ? std::atoi(argv[4]) : 0);
    if (argc >= 4 && !std::strcmp(argv[1], "imgdump")) return imgdump(argv[2], argv[3]);
    if (argc >= 5 && !std::strcmp(argv[1], "dumpavg"))
        return dumpavg(argv[2], argv[3], std::atoi(argv[4]), argc > 5 ? std::atoi(argv[5]) : 0);
    if (argc >= 5 && !std::strcmp(argv[1], "bench"))
        return bench(argv[2], std::atoi(argv[3]), std::atoi(argv[4]), argc > 5 ? std::atoi(argv[5]) : 0,
                     argc > 6 ? argv[6] : "refdriver_bench.png", argc > 8 ? std::atoi(argv[7]) : 0,
                     argc > 8 ? std::atoi(argv[8]) : 0);
    std::fprintf(stderr, "usage: refdriver dump <scene.xml> <out.bin> [camera] | bench <scene.xml> <threads> <reps> [camera]\n");
    return 2;
}
