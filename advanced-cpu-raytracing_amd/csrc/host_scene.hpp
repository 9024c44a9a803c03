#pragma once

#include <string>
#include <vector>

#include "host_math.hpp"
#include "rtgpu.h"

namespace rtg {

// Owner of every array an rtg_scene_desc points into.
struct HostScene {
    struct ImageStore {
        int id = 0, width = 0, height = 0, channels = 0, is_hdr = 0;
        std::vector<float> texels;
    };
    int background[3] = {0, 0, 0};
    float shadowEps = 0.001f;
    int maxDepth = 0;
    int bgTexture = -1;
    bool motionBlurEnabled = false;
    std::vector<rtg_mesh_light> mesh_lights;
    bool deferBvh = false;      // RTG_LOAD_DEVICE_BVH: faces in parse order, no BVH (built on the device)
    V3 ambient;
    std::vector<rtg_camera> cameras;
    std::vector<rtg_material> materials;
    std::vector<rtg_brdf> brdfs;
    std::vector<rtg_point_light> point_lights;
    std::vector<rtg_area_light> area_lights;
    std::vector<rtg_directional_light> dir_lights;
    std::vector<rtg_spot_light> spot_lights;
    std::vector<rtg_env_light> env_lights;
    std::vector<rtg_texture> textures;
    std::vector<ImageStore> imageStore;
    std::vector<rtg_image> images;
    std::vector<rtg_object> objects;
    std::vector<rtg_mesh> meshes;
    std::vector<rtg_face> faces;
    std::vector<rtg_bvh_node> nodes;
    rtg_scene_desc desc;

    int load(const std::string& xml_path, std::string& err);
    void finalize();
};

}  // namespace rtg

struct rtg_host_scene {
    rtg::HostScene s;
};
