// Adapter: the reference's own object model (DorkTracer::Scene after Scene::loadFromXml,
// src/scene.h:32-89, built by its tinyxml2 parser src/parser.cpp) -> the flat POD
// rtg_scene_desc of include/rtgpu.h.  This is the drop-in north_star asks for: the reference
// keeps its parser, Scene / Camera / Material / Light objects and CLI, and hands the scene to
// librtgpu through this one function instead of constructing a Raytracer (raytracer.cpp:7-16).
//
// Built only where the reference sources are (integration/Makefile compiles against
// /root/reference/src and links the reference's objects from oracle/_ref); nothing of the
// reference is copied into this repository.
#pragma once

#include <string>
#include <vector>

#include "rtgpu.h"

namespace DorkTracer {
class Scene;
}

namespace rtg_dork {

// Owner of every array the description points into.
struct DescOwner {
    std::vector<rtg_camera> cameras;
    std::vector<rtg_material> materials;
    std::vector<rtg_brdf> brdfs;
    std::vector<rtg_point_light> point_lights;
    std::vector<rtg_area_light> area_lights;
    std::vector<rtg_directional_light> dir_lights;
    std::vector<rtg_spot_light> spot_lights;
    std::vector<rtg_env_light> env_lights;
    std::vector<rtg_texture> textures;
    std::vector<std::vector<float>> texels;
    std::vector<rtg_image> images;
    std::vector<rtg_object> objects;
    std::vector<rtg_mesh> meshes;
    std::vector<rtg_face> faces;
    std::vector<rtg_bvh_node> nodes;
    std::vector<rtg_mesh_light> mesh_lights;
    rtg_scene_desc desc;
};

// Fills `out` from a loaded reference scene.  Returns RTG_OK or a negative rtg_status with a
// message in `err` (features the GPU path does not take: EXR images).
int desc_from_scene(DorkTracer::Scene& scene, DescOwner& out, std::string& err);

}  // namespace rtg_dork
