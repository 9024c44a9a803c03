// DorkTracer::Scene -> rtg_scene_desc (see dork_adapter.hpp).
//
// The reference keeps a few fields the description needs behind `private` / `protected`
// (Camera::m_q and the image-plane extents camera.hpp:44-46, its tonemapper and renderer
// params, AreaLight's basis, SpotLight's cosines, Mesh's vertex / uv arrays, the instance's
// material id, texture internals, LDRImage's channel count).  This one translation unit opens
// them by defining the access keywords away before including the reference's headers (the
// standard library is included first, untouched); the class layouts do not change, and the
// reference's own objects -- compiled without it -- are what is read.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <iostream>
#include <limits>
#include <map>
#include <random>
#include <sstream>
#include <string>
#include <vector>

#define private public
#define protected public
#include "scene.h"
#include "instancedMesh.hpp"
#include "imageTexture.h"
#include "perlinTexture.h"
#include "LDRImage.h"
#include "HDRImage.h"
#include "brdfBlinnPhong.h"
#include "brdfModifiedBlinnPhong.h"
#include "brdfModifiedPhong.h"
#include "brdfPhong.h"
#include "brdfTorranceSparrow.h"
#undef private
#undef protected

#include "dork_adapter.hpp"

using namespace DorkTracer;

namespace rtg_dork {
namespace {

rtg_float3 f3(const Vec3f& v) { return rtg_float3{v.x, v.y, v.z}; }

void mat16(Matrix& m, double* out) {
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c) out[4 * r + c] = (m.row == 4 && m.col == 4) ? m[r][c] : 0.0;
}

template <typename T>
int index_of(const std::vector<T*>& v, const void* p) {
    for (size_t i = 0; i < v.size(); ++i)
        if ((const void*)v[i] == p) return (int)i;
    return -1;
}

}  // namespace

int desc_from_scene(Scene& S, DescOwner& D, std::string& err) {
    D = DescOwner();
    // ---- cameras (camera.hpp:15-50; one Camera object reused by the parser, parser.cpp:1504)
    for (Camera& c : S.cameras) {
        rtg_camera o;
        std::memset(&o, 0, sizeof(o));
        o.position = f3(c.position); o.gaze = f3(c.gaze); o.up = f3(c.up); o.right = f3(c.right); o.q = f3(c.m_q);
        o.left = c.m_left; o.right_ext = c.m_right; o.bottom = c.m_bottom; o.top = c.m_top;
        o.near_dist = c.nearDist;
        o.width = c.imageWidth; o.height = c.imageHeight; o.spp = c.samplesPerPixel;
        o.focus_distance = c.focusDistance; o.aperture = c.apertureSize;
        o.has_tonemapper = c.hasTonemapper;
        if (c.hasTonemapper && c.tonemapper) {
            o.tm_key = c.tonemapper->keyValue; o.tm_burn = c.tonemapper->burnPerct;
            o.tm_saturation = c.tonemapper->saturation; o.tm_gamma = c.tonemapper->gamma;
        }
        RendererParams& rp = c.rendererParams;
        o.path_tracing = rp.pathTracingEnabled; o.importance_sampling = rp.sampleImportance;
        o.next_event = rp.nextEventEstimationEnabled; o.russian_roulette = rp.russianRouletteEnabled;
        std::strncpy(o.image_name, c.imageName.c_str(), sizeof(o.image_name) - 1);
        D.cameras.push_back(o);
    }
    // ---- BRDFs (brdf*.h), in scene.brdfs order
    for (BRDF* b : S.brdfs) {
        rtg_brdf o;
        std::memset(&o, 0, sizeof(o));
        o.id = b->id;
        o.exponent = b->exponent;
        o.energy_conserving = b->isEnergyConserving;
        if (dynamic_cast<BrdfModifiedBlinnPhong*>(b)) o.type = RTG_BRDF_MODIFIED_BLINN_PHONG;
        else if (dynamic_cast<BrdfBlinnPhong*>(b)) o.type = RTG_BRDF_BLINN_PHONG;
        else if (dynamic_cast<BrdfModifiedPhong*>(b)) o.type = RTG_BRDF_MODIFIED_PHONG;
        else if (dynamic_cast<BrdfPhong*>(b)) o.type = RTG_BRDF_PHONG;
        else if (auto* ts = dynamic_cast<BrdfTorranceSparrow*>(b)) {
            o.type = RTG_BRDF_TORRANCE_SPARROW;
            o.kd_fresnel = ts->kdFresnel;
        }
        D.brdfs.push_back(o);
    }
    // ---- materials (material.hpp:8-48; matId - 1 indexes them, raytracer.cpp:73)
    for (Material& m : S.materials) {
        rtg_material o;
        std::memset(&o, 0, sizeof(o));
        o.id = m.id;
        o.type = (int32_t)m.type;
        o.brdf = m.brdf ? index_of(S.brdfs, m.brdf) : -1;
        o.ambient = f3(m.ambient); o.diffuse = f3(m.diffuse); o.specular = f3(m.specular); o.mirror = f3(m.mirror);
        o.phong_exponent = m.phong_exponent;
        o.refractive_index = m.refractiveIndex;
        o.absorption_index = m.conductorAbsorptionIndex;
        o.roughness = m.roughness;
        o.absorption = f3(m.absorptionCoefficient);
        o.radiance = f3(m.radiance);
        D.materials.push_back(o);
    }
    // ---- lights, in SampleDirectLighting's type order (raytracer.cpp:706-803)
    for (PointLight& l : S.point_lights) D.point_lights.push_back(rtg_point_light{f3(l.position), f3(l.intensity)});
    for (AreaLight* l : S.areaLights) {
        rtg_area_light o;
        o.position = f3(l->position); o.normal = f3(l->normal); o.radiance = f3(l->radiance);
        o.u = f3(l->u); o.v = f3(l->v);
        o.extent = l->extent; o.area = l->area;
        D.area_lights.push_back(o);
    }
    for (DirectionalLight* l : S.directionalLights) D.dir_lights.push_back(rtg_directional_light{f3(l->dir), f3(l->radiance)});
    for (SpotLight* l : S.spotLights) {
        rtg_spot_light o;
        std::memset(&o, 0, sizeof(o));
        o.position = f3(l->pos); o.dir = f3(l->dir); o.intensity = f3(l->intensity);
        o.coverage_deg = l->coverageAngle; o.falloff_deg = l->falloffAngle;
        o.cos_half_coverage = l->cosHalfCoverage; o.cos_half_falloff = l->cosHalfFalloff;
        D.spot_lights.push_back(o);
    }
    // ---- images (LDRImage.h: raw 0..255 bytes; HDRImage.h: LoadEXR's R, G, B floats)
    for (Image* im : S.images) {
        rtg_image o;
        std::memset(&o, 0, sizeof(o));
        if (auto* ldr = dynamic_cast<LDRImage*>(im)) {
            const size_t n = (size_t)ldr->width * ldr->height * ldr->channels;
            D.texels.emplace_back(ldr->image, ldr->image + n);
            o.id = ldr->id; o.width = ldr->width; o.height = ldr->height; o.channels = ldr->channels;
        } else if (auto* hdr = dynamic_cast<HDRImage*>(im)) {
            D.texels.emplace_back(hdr->src.begin(), hdr->src.end());
            o.id = hdr->id; o.width = hdr->width; o.height = hdr->height; o.channels = 3;
            o.is_hdr = 1;
        } else {
            err = "image " + std::to_string(im->id) + ": unknown image class";
            return RTG_ERR_UNSUPPORTED;
        }
        D.images.push_back(o);
    }
    for (size_t i = 0; i < D.images.size(); ++i) D.images[i].texels = D.texels[i].data();
    for (SphericalEnvironmentLight* l : S.sphericalEnvLights) {
        rtg_env_light o;
        std::memset(&o, 0, sizeof(o));
        o.image = index_of(S.images, l->image);
        D.env_lights.push_back(o);
    }
    // ---- textures (texture.h, imageTexture.h, perlinTexture.h)
    for (Texture* t : S.textures) {
        rtg_texture o;
        std::memset(&o, 0, sizeof(o));
        o.id = t->id;
        o.is_background = t == S.bgTexture;
        o.slot = o.is_background ? RTG_TEXSLOT_NONE : (int32_t)t->type;   // Diffuse .. ReplaceAll = the slots
        o.blend = !o.is_background && t->operationMode == Texture::Blend && t->type == Texture::Textures::Diffuse;
        o.image = -1;
        if (auto* it = dynamic_cast<ImageTexture*>(t)) {
            o.kind = RTG_TEX_IMAGE;
            o.image = index_of(S.images, it->img);
            o.nearest = it->interpolationMode == ImageTexture::InterpolationMode::Nearest;
            o.normalizer = it->normalizer;
            o.bump_factor = it->sampleMultiplier;
        } else if (auto* pt = dynamic_cast<PerlinTexture*>(t)) {
            o.kind = RTG_TEX_PERLIN;
            o.noise_scale = pt->scale;
            o.noise_abs = pt->conversionType == PerlinTexture::Conversion::AbsoluteVal;
            o.bump_factor = pt->bumpFactor;
            o.normalizer = 1.0f;
        }
        D.textures.push_back(o);
    }
    auto tex = [&](Texture* t) { return t ? index_of(S.textures, t) : -1; };
    // ---- geometry: every non-instance Mesh of scene.meshes (Mesh, LightMesh, Triangle),
    // its faces in BVH-permuted order and its BVH nodes (mesh.cpp:23-156)
    std::map<const Mesh*, int> meshIndex;
    for (Shape* s : S.meshes) {
        if (s->isInstance) continue;
        Mesh* m = static_cast<Mesh*>(s);
        rtg_mesh o;
        std::memset(&o, 0, sizeof(o));
        o.face_offset = (int32_t)D.faces.size();
        o.face_count = (int32_t)m->faces.size();
        o.node_offset = (int32_t)D.nodes.size();
        o.node_count = (int32_t)m->nextFreeNodeIdx;
        o.has_uv = m->uv.empty() ? 0 : 1;
        // Mesh::surfaceArea is never initialised by the reference (mesh.cpp:7-13; parser.cpp:608
        // adds every face's area to it): the sum of the face areas, its evident intent -- summed
        // here in BVH order, so it may differ from rtg_host_scene_load_xml's parse-order sum in
        // the last bits (dorkrt --compare allows that, and only that)
        o.surface_area = 0.0;
        for (Face& f : m->faces) o.surface_area += f.area;
        for (Face& f : m->faces) {
            rtg_face r;
            std::memset(&r, 0, sizeof(r));
            r.v0 = f3(m->GetVertex(f.v0_id)); r.v1 = f3(m->GetVertex(f.v1_id)); r.v2 = f3(m->GetVertex(f.v2_id));
            r.n = f3(f.n);
            if (o.has_uv) {
                const Vec2f a = m->GetUv(f.v0_id), b = m->GetUv(f.v1_id), c = m->GetUv(f.v2_id);
                r.uv0[0] = a.x; r.uv0[1] = a.y; r.uv1[0] = b.x; r.uv1[1] = b.y; r.uv2[0] = c.x; r.uv2[1] = c.y;
            }
            r.area = f.area;
            D.faces.push_back(r);
        }
        for (uint32_t k = 0; k < m->nextFreeNodeIdx; ++k) {
            BVH& b = m->bvh[k];
            rtg_bvh_node n;
            std::memset(&n, 0, sizeof(n));
            n.bmin[0] = b.bbox.minCorner.x; n.bmin[1] = b.bbox.minCorner.y; n.bmin[2] = b.bbox.minCorner.z;
            n.bmax[0] = b.bbox.maxCorner.x; n.bmax[1] = b.bbox.maxCorner.y; n.bmax[2] = b.bbox.maxCorner.z;
            n.left = b.left ? (int32_t)(b.left - &m->bvh[0]) : -1;
            n.first = (int32_t)b.firstFace;
            n.count = b.left ? 0 : (int32_t)b.faceCount;
            D.nodes.push_back(n);
        }
        meshIndex[m] = (int)D.meshes.size();
        D.meshes.push_back(o);
    }
    // ---- objects in IntersectObjects order (raytracer.cpp:625-643): scene.meshes, spheres
    for (Shape* s : S.meshes) {
        rtg_object o;
        std::memset(&o, 0, sizeof(o));
        Mesh* geo;
        if (s->isInstance) {
            auto* im = static_cast<InstancedMesh*>(s);
            geo = im->baseMesh;
            o.kind = RTG_OBJ_INSTANCE;
            // InstancedMesh::SetMaterial writes its own member (instancedMesh.hpp:23), not
            // Shape::material_id: the instance's material is that member
            o.material = im->material_id - 1;
            mat16(geo->inverseTransposeTransform, o.base_inv_transpose);
            o.bbox_min[0] = im->bbox.minCorner.x; o.bbox_min[1] = im->bbox.minCorner.y; o.bbox_min[2] = im->bbox.minCorner.z;
            o.bbox_max[0] = im->bbox.maxCorner.x; o.bbox_max[1] = im->bbox.maxCorner.y; o.bbox_max[2] = im->bbox.maxCorner.z;
        } else {
            geo = static_cast<Mesh*>(s);
            o.kind = RTG_OBJ_MESH;
            o.material = s->material_id - 1;
            mat16(s->inverseTransposeTransform, o.base_inv_transpose);
            o.bbox_min[0] = geo->bbox.minCorner.x; o.bbox_min[1] = geo->bbox.minCorner.y; o.bbox_min[2] = geo->bbox.minCorner.z;
            o.bbox_max[0] = geo->bbox.maxCorner.x; o.bbox_max[1] = geo->bbox.maxCorner.y; o.bbox_max[2] = geo->bbox.maxCorner.z;
        }
        if (o.material < 0 || o.material >= (int)S.materials.size()) {
            err = "mesh " + std::to_string(s->id) + ": material out of range";
            return RTG_ERR_INVALID;
        }
        o.mesh = meshIndex.at(geo);
        o.id = s->id;
        if (S.materials[o.material].type == Material::Emissive) o.flags |= RTG_OBJF_SHADOW_SKIP;
        if (geo->uv.empty()) o.flags |= RTG_OBJF_NORMAL_TWICE;
        if (s->hasMotionBlur) o.flags |= RTG_OBJF_MOTION_BLUR;
        o.tex_diffuse = tex(s->diffuseTex); o.tex_specular = tex(s->specularTex); o.tex_replace_all = tex(s->replaceAll);
        // normal / bump maps are read by the base Mesh's IntersectFace (mesh.cpp:263-358)
        o.tex_normal = tex(geo->normalMap); o.tex_bump = tex(geo->bumpMap);
        mat16(s->inverseTransform, o.inv_transform);
        mat16(s->inverseTransposeTransform, o.inv_transpose);
        mat16(s->transform, o.transform);
        o.motion_blur = f3(s->motionBlurVector);
        D.objects.push_back(o);
    }
    for (Sphere* sp : S.spheres) {
        rtg_object o;
        std::memset(&o, 0, sizeof(o));
        o.kind = RTG_OBJ_SPHERE;
        o.material = sp->material_id - 1;         // Sphere's own member shadows Shape's (sphere.hpp:13)
        if (o.material < 0 || o.material >= (int)S.materials.size()) {
            err = "sphere: material out of range";
            return RTG_ERR_INVALID;
        }
        o.mesh = -1;
        if (sp->hasMotionBlur) o.flags |= RTG_OBJF_MOTION_BLUR;
        o.tex_diffuse = tex(sp->diffuseTex); o.tex_specular = tex(sp->specularTex); o.tex_normal = tex(sp->normalMap);
        o.tex_bump = tex(sp->bumpMap); o.tex_replace_all = tex(sp->replaceAll);
        mat16(sp->inverseTransform, o.inv_transform);
        mat16(sp->inverseTransposeTransform, o.inv_transpose);
        mat16(sp->inverseTransposeTransform, o.base_inv_transpose);
        mat16(sp->transform, o.transform);
        if (sp->center_vertex_id < 1 || sp->center_vertex_id > (int)sp->vertex_data.size()) {
            err = "sphere: center vertex out of range";
            return RTG_ERR_INVALID;
        }
        o.center = f3(sp->vertex_data[sp->center_vertex_id - 1]);
        o.radius = sp->radius;
        o.motion_blur = f3(sp->motionBlurVector);
        D.objects.push_back(o);
    }
    // ---- mesh lights (meshLight.h), scene.meshLights order; object = its slot in scene.meshes
    for (MeshLight* ml : S.meshLights) {
        rtg_mesh_light o;
        std::memset(&o, 0, sizeof(o));
        o.object = index_of(S.meshes, static_cast<Shape*>(ml));
        o.radiance = f3(ml->radiance);
        D.mesh_lights.push_back(o);
    }
    // ---- the description
    rtg_scene_desc& d = D.desc;
    std::memset(&d, 0, sizeof(d));
    d.background[0] = S.background_color.x; d.background[1] = S.background_color.y; d.background[2] = S.background_color.z;
    d.shadow_epsilon = Scene::shadow_ray_epsilon;
    d.max_recursion_depth = S.max_recursion_depth;
    d.bg_texture = S.bgTexture ? index_of(S.textures, S.bgTexture) : -1;
    d.ambient_light = f3(S.ambient_light);
    d.cameras = D.cameras.data(); d.num_cameras = (int32_t)D.cameras.size();
    d.materials = D.materials.data(); d.num_materials = (int32_t)D.materials.size();
    d.brdfs = D.brdfs.data(); d.num_brdfs = (int32_t)D.brdfs.size();
    d.point_lights = D.point_lights.data(); d.num_point_lights = (int32_t)D.point_lights.size();
    d.area_lights = D.area_lights.data(); d.num_area_lights = (int32_t)D.area_lights.size();
    d.dir_lights = D.dir_lights.data(); d.num_dir_lights = (int32_t)D.dir_lights.size();
    d.spot_lights = D.spot_lights.data(); d.num_spot_lights = (int32_t)D.spot_lights.size();
    d.env_lights = D.env_lights.data(); d.num_env_lights = (int32_t)D.env_lights.size();
    d.textures = D.textures.data(); d.num_textures = (int32_t)D.textures.size();
    d.images = D.images.data(); d.num_images = (int32_t)D.images.size();
    d.objects = D.objects.data(); d.num_objects = (int32_t)D.objects.size();
    d.meshes = D.meshes.data(); d.num_meshes = (int32_t)D.meshes.size();
    d.faces = D.faces.data(); d.num_faces = (int64_t)D.faces.size();
    d.nodes = D.nodes.data(); d.num_nodes = (int64_t)D.nodes.size();
    d.mesh_lights = D.mesh_lights.data(); d.num_mesh_lights = (int32_t)D.mesh_lights.size();
    return RTG_OK;
}

}  // namespace rtg_dork
