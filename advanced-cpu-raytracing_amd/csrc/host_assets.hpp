#pragma once

#include <array>
#include <string>
#include <vector>

namespace rtg {

struct PlyData {
    std::vector<std::array<double, 3>> positions;   // happly getVertexPositions()
    std::vector<std::vector<int>> faces;            // happly getFaceIndices<int>()
};
bool load_ply(const std::string& path, PlyData& out, std::string& err);

struct Image8 {
    int width = 0, height = 0, channels = 0;
    std::vector<unsigned char> data;
};
bool load_image8(const std::string& path, Image8& img, std::string& err);
// HDRImage (HDRImage.h:45-72): LoadEXR's RGBA, alpha dropped -> width*height*3 floats
bool load_exr(const std::string& path, int& width, int& height, std::vector<float>& rgb, std::string& err);

bool write_png(const std::string& path, int w, int h, const unsigned char* rgb, std::string& err);
bool write_hdr(const std::string& path, int w, int h, const float* rgb, std::string& err);

}  // namespace rtg
