// XML scene loader -> rtg_scene_desc.
//
// Follows DorkTracer::Scene::loadFromXml (src/parser.cpp:26-577) and its helpers
// statement by statement, including the behaviours the rendered pixels depend on:
//   * one std::stringstream per parse function, values carried across elements
//     (RefStream, host_xml.hpp);
//   * ONE Material object reused for every <Material> (parser.cpp:1115): brdf,
//     ambient, diffuse and specular are inherited when absent;
//   * ONE Camera object reused for every <Camera> (parser.cpp:1504): tonemapper and
//     renderer params are inherited;
//   * mesh bounding boxes start at max = FLT_MIN (parser.cpp:1393);
//   * meshes without UVs get their normal transformed twice (mesh.cpp:362 + :179);
//   * the midpoint-split BVH with in-place face partition (mesh.cpp:23-156),
//     reproduced exactly so face order / node topology match the reference;
//   * single-character transform ids (parser.cpp:663,689,699).
#include <cfloat>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <limits>
#include <stdexcept>
#include <string>
#include <vector>

#include "host_assets.hpp"
#include "host_math.hpp"
#include "host_scene.hpp"
#include "host_xml.hpp"

namespace rtg {

namespace {

struct LoadError : std::runtime_error {
    int code;
    LoadError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};
[[noreturn]] void fail(int code, const std::string& msg) { throw LoadError(code, msg); }

struct BBox { V3 mn, mx; };

struct FaceRec {              // shape.hpp:103-112
    int v0, v1, v2;
    V3 n, center;
    BBox bbox;
    double area;
};

struct Geometry {             // a Mesh's geometry (mesh.hpp)
    std::vector<V3> verts;
    std::vector<std::array<float, 2>> uv;
    int vertexOffset = 0, textureOffset = 0;
    std::vector<FaceRec> faces;
    BBox bbox;
    double surfaceArea = 0.0;
    const V3& vertex(int idx) const {                     // mesh.cpp:19-21
        long k = (long)idx - 1 + vertexOffset;
        if (k < 0 || k >= (long)verts.size()) fail(RTG_ERR_PARSE, "vertex index out of range");
        return verts[k];
    }
    std::array<float, 2> texcoord(int idx) const {        // mesh.cpp:16-18
        long k = (long)idx - 1 + textureOffset;
        if (k < 0 || k >= (long)uv.size()) fail(RTG_ERR_PARSE, "texture coordinate index out of range");
        return uv[k];
    }
};

struct Xform { M4 transform, inverse, invTranspose; };

struct ShapeRec {             // an entry of scene.meshes (Mesh, LightMesh, MeshInstance, Triangle)
    int id = 0;
    bool isInstance = false;
    int geometry = -1;        // geometry of the (root) base mesh for instances
    int parentShape = -1;     // instances: immediate parent in scene.meshes
    int material = 0;         // 1-based as in the XML
    int tex[5] = {-1, -1, -1, -1, -1};   // diffuse, specular, normal, bump, replace_all
    Xform xf;
    BBox bbox;                // instances: world bbox
    bool motionBlur = false;
    V3 mbv;
    bool lightMesh = false;
};

struct SphereRec {
    int material = 0;
    int centerId = 0;
    float radius = 0.f;
    int tex[5] = {-1, -1, -1, -1, -1};
    Xform xf;
    bool motionBlur = false;
    V3 mbv;
};

struct TexRec {
    rtg_texture t;
    std::string decal;
};

class Loader {
public:
    explicit Loader(HostScene& out) : S(out) {}
    void load(const std::string& path);

private:
    HostScene& S;
    std::vector<V3> vertex_data;
    std::vector<std::array<float, 2>> texCoords;
    std::vector<V3> translations, scalings;
    struct Rot { float w, x, y, z; };
    std::vector<Rot> rotations;
    std::vector<Geometry> geos;
    std::vector<ShapeRec> shapes;   // scene.meshes order
    std::vector<SphereRec> spheres;
    std::vector<TexRec> texs;
    std::vector<int> imageIds;

    void parseCameras(XmlNode* root);
    void parseLights(XmlNode* root);
    void parseBRDFs(XmlNode* root);
    void parseMaterials(XmlNode* root);
    void parseTextures(XmlNode* root, RefStream& stream);
    void parseMeshes(XmlNode* root, const char* elemName);
    void setupTextures(int* tex, std::string ids);
    void computeTransform(Xform& xf, const std::string& input);
    void computeFaceProperties(FaceRec& f, Geometry& g);
    void constructBVH(Geometry& g, std::vector<rtg_bvh_node>& nodes);
    BBox transformBoundingBox(const BBox& b, const M4& t);
    void flatten();
    std::chrono::steady_clock::time_point tStart;
    double bvhSeconds = 0.0;
};

std::string need_text(XmlNode* e, const char* what) {
    if (!e) fail(RTG_ERR_PARSE, std::string("missing <") + what + ">");
    const char* t = e->GetText();
    if (!t) fail(RTG_ERR_PARSE, std::string("empty <") + what + ">");
    return t;
}

// ---------------------------------------------------------------------------
void Loader::load(const std::string& path) {
    tStart = std::chrono::steady_clock::now();
    XmlDocument file;
    if (!file.Load(path))
        fail(file.error.rfind("cannot open", 0) == 0 ? RTG_ERR_IO : RTG_ERR_PARSE,
             "Error: The xml file cannot be loaded. " + file.error);
    XmlNode* root = file.FirstChild();
    if (!root) fail(RTG_ERR_PARSE, "Error: Root is not found.");

    RefStream stream;
    XmlNode *child, *element;
    S.motionBlurEnabled = false;

    // parser.cpp:46-70
    int bg[3] = {0, 0, 0};
    element = root->FirstChildElement("BackgroundColor");
    if (element) { stream.line(element->GetText()); stream.get(bg[0]).get(bg[1]).get(bg[2]); }
    std::memcpy(S.background, bg, sizeof(bg));
    S.shadowEps = 0.001f;   // scene.cpp:3 (static; re-initialised per load here)
    element = root->FirstChildElement("ShadowRayEpsilon");
    if (element) { stream.line(element->GetText()); stream.get(S.shadowEps); }
    S.maxDepth = 0;
    element = root->FirstChildElement("MaxRecursionDepth");
    if (element) { stream.line(element->GetText()); stream.get(S.maxDepth); }

    parseCameras(root);
    parseLights(root);
    parseBRDFs(root);
    parseMaterials(root);

    S.bgTexture = -1;
    parseTextures(root, stream);

    // environment lights after images (parser.cpp:231-261)
    element = root->FirstChildElement("Lights");
    if (element) {
        element = element->FirstChildElement("SphericalDirectionalLight");
        while (element) {
            int id = 0, imageId = 0;
            stream.line(element->Attribute("id")); stream.get(id);
            child = element->FirstChildElement("ImageId");
            stream.line(child ? child->GetText() : nullptr); stream.get(imageId);
            int img = -1;
            for (size_t i = 0; i < imageIds.size(); ++i) if (imageIds[i] == imageId) { img = (int)i; break; }
            if (img < 0) fail(RTG_ERR_PARSE, "SphericalDirectionalLight: no image with id " + std::to_string(imageId));
            rtg_env_light el; el.image = img; el.pad0 = 0;
            S.env_lights.push_back(el);
            element = element->NextSiblingElement("SphericalDirectionalLight");
        }
        stream.clear();
    }

    // VertexData (parser.cpp:264-277)
    element = root->FirstChildElement("VertexData");
    if (element) {
        stream.line(element->GetText());
        V3 v;
        while (!stream.get(v.x).eof()) {
            stream.get(v.y).get(v.z);
            vertex_data.push_back(v);
            if (stream.fail() && !stream.eof()) fail(RTG_ERR_PARSE, "malformed <VertexData>");
        }
    }
    stream.clear();

    // TexCoordData (parser.cpp:279-291).  An empty element makes the reference loop
    // forever; report it instead.
    element = root->FirstChildElement("TexCoordData");
    if (element) {
        if (!element->GetText()) fail(RTG_ERR_PARSE, "empty <TexCoordData/> (the reference parser loops forever on it)");
        stream.line(element->GetText());
        std::array<float, 2> tc;
        while (!stream.get(tc[0]).eof()) {
            stream.get(tc[1]);
            texCoords.push_back(tc);
            if (stream.fail() && !stream.eof()) fail(RTG_ERR_PARSE, "malformed <TexCoordData>");
        }
        stream.clear();
    }

    // Transformations (parser.cpp:293-345)
    element = root->FirstChildElement("Transformations");
    if (element) {
        for (XmlNode* c = element->FirstChildElement("Translation"); c; c = c->NextSiblingElement("Translation")) {
            if (!c->Attribute("id")) fail(RTG_ERR_PARSE, "Translation without id");
            stream.line(c->GetText());
            V3 t; stream.get(t.x).get(t.y).get(t.z);
            translations.push_back(t);
        }
        for (XmlNode* c = element->FirstChildElement("Scaling"); c; c = c->NextSiblingElement("Scaling")) {
            if (!c->Attribute("id")) fail(RTG_ERR_PARSE, "Scaling without id");
            stream.line(c->GetText());
            V3 s; stream.get(s.x).get(s.y).get(s.z);
            scalings.push_back(s);
        }
        for (XmlNode* c = element->FirstChildElement("Rotation"); c; c = c->NextSiblingElement("Rotation")) {
            if (!c->Attribute("id")) fail(RTG_ERR_PARSE, "Rotation without id");
            stream.line(c->GetText());
            Rot r; stream.get(r.w).get(r.x).get(r.y).get(r.z);
            rotations.push_back(r);
        }
    }
    stream.clear();

    parseMeshes(root, "Mesh");
    parseMeshes(root, "LightMesh");

    XmlNode* objects = root->FirstChildElement("Objects");
    if (!objects) fail(RTG_ERR_PARSE, "missing <Objects>");

    // MeshInstance (parser.cpp:352-455)
    for (element = objects->FirstChildElement("MeshInstance"); element;
         element = element->NextSiblingElement("MeshInstance")) {
        bool resetTransform = false;
        if (const char* rt = element->Attribute("resetTransform")) resetTransform = std::string(rt) == "true";
        int ownId = 0, baseMeshId = 0;
        stream.line(element->Attribute("id")); stream.get(ownId);
        stream.line(element->Attribute("baseMeshId")); stream.get(baseMeshId);
        int parent = -1;
        for (size_t i = 0; i < shapes.size(); ++i)
            if (shapes[i].id == baseMeshId) parent = (int)i;     // last match wins (no break)
        if (parent < 0) fail(RTG_ERR_PARSE, "MeshInstance: no base mesh with id " + std::to_string(baseMeshId));
        int base = parent;
        while (shapes[base].isInstance) base = shapes[base].parentShape >= 0 ? shapes[base].parentShape : base;
        ShapeRec inst;
        inst.id = ownId;
        inst.isInstance = true;
        inst.geometry = shapes[base].geometry;
        inst.parentShape = base;      // resolved root base mesh (instancedMesh baseMesh)
        child = element->FirstChildElement("Textures");
        if (child) setupTextures(inst.tex, need_text(child, "Textures") + " ");
        child = element->FirstChildElement("Material");
        if (child) {
            stream.line(child->GetText());
            int matId = 0;
            stream.get(matId);
            inst.material = matId;
        } else {
            inst.material = shapes[base].material;
        }
        child = element->FirstChildElement("MotionBlur");
        if (child) {
            stream.line(child->GetText());
            stream.get(inst.mbv.x).get(inst.mbv.y).get(inst.mbv.z);
            S.motionBlurEnabled = true;
            inst.motionBlur = true;
        }
        child = element->FirstChildElement("Transformations");
        inst.xf.transform = M4::identity();
        inst.xf.inverse = M4::identity();
        inst.xf.invTranspose = M4::zero();     // Shape() leaves it zero (shape.hpp:72); only set below
        if (child) {
            computeTransform(inst.xf, need_text(child, "Transformations"));
            if (!resetTransform) {
                const Xform& px = shapes[parent].xf;
                inst.xf.transform = inst.xf.transform * px.transform;
                inst.xf.inverse = px.inverse * inst.xf.inverse;
                inst.xf.invTranspose = inst.xf.inverse.transpose();
            }
        }
        inst.bbox = transformBoundingBox(geos[inst.geometry].bbox, inst.xf.transform);
        shapes.push_back(inst);
    }

    // Triangles as 1-face meshes (parser.cpp:458-512)
    for (element = objects->FirstChildElement("Triangle"); element;
         element = element->NextSiblingElement("Triangle")) {
        Geometry g;
        g.verts = vertex_data;
        g.uv = texCoords;
        ShapeRec sh;
        child = element->FirstChildElement("Transformations");
        sh.xf.transform = M4::identity();
        sh.xf.inverse = M4::identity();
        sh.xf.invTranspose = M4::identity();
        if (child) computeTransform(sh.xf, need_text(child, "Transformations"));
        child = element->FirstChildElement("Textures");
        if (child) setupTextures(sh.tex, need_text(child, "Textures") + " ");
        child = element->FirstChildElement("Material");
        stream.line(child ? child->GetText() : nullptr);
        int matId = 0;
        stream.get(matId);
        sh.material = matId;
        child = element->FirstChildElement("Indices");
        stream.line(child ? child->GetText() : nullptr);
        FaceRec f;
        stream.get(f.v0).get(f.v1).get(f.v2);
        computeFaceProperties(f, g);
        g.faces.push_back(f);
        g.bbox = f.bbox;
        sh.id = 0;   // Shape::id is never assigned for triangles
        sh.geometry = (int)geos.size();
        geos.push_back(std::move(g));
        shapes.push_back(sh);
    }

    // Spheres (parser.cpp:514-574)
    for (element = objects->FirstChildElement("Sphere"); element; element = element->NextSiblingElement("Sphere")) {
        SphereRec sp;
        child = element->FirstChildElement("Transformations");
        sp.xf.transform = M4::identity();
        sp.xf.inverse = M4::identity();
        sp.xf.invTranspose = M4::identity();
        if (child) computeTransform(sp.xf, need_text(child, "Transformations"));
        child = element->FirstChildElement("Textures");
        if (child) setupTextures(sp.tex, need_text(child, "Textures") + " ");
        child = element->FirstChildElement("Material");
        stream.line(child ? child->GetText() : nullptr); stream.get(sp.material);
        child = element->FirstChildElement("Center");
        stream.line(child ? child->GetText() : nullptr); stream.get(sp.centerId);
        child = element->FirstChildElement("Radius");
        stream.line(child ? child->GetText() : nullptr); stream.get(sp.radius);
        child = element->FirstChildElement("MotionBlur");
        if (child) {
            stream.line(child->GetText());
            stream.get(sp.mbv.x).get(sp.mbv.y).get(sp.mbv.z);
            sp.motionBlur = true;
            S.motionBlurEnabled = true;
        }
        spheres.push_back(sp);
    }

    const auto t0 = std::chrono::steady_clock::now();
    flatten();
    if (std::getenv("RTG_HOST_TIMING")) {   // ingest phase timings (DESIGN.md measurements)
        const auto t1 = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[rtg host] parse+faces %.3f s, bvh build %.3f s, flatten %.3f s\n",
                     std::chrono::duration<double>(t0 - tStart).count(), bvhSeconds,
                     std::chrono::duration<double>(t1 - t0).count());
    }
}

// ---------------------------------------------------------------------------
void Loader::parseCameras(XmlNode* root) {            // parser.cpp:1498-1636
    XmlNode* cams = root->FirstChildElement("Cameras");
    if (!cams) fail(RTG_ERR_PARSE, "missing <Cameras>");
    RefStream stream;
    rtg_camera cam;                                    // reused across cameras (parser.cpp:1504)
    std::memset(&cam, 0, sizeof(cam));
    for (XmlNode* element = cams->FirstChildElement("Camera"); element;
         element = element->NextSiblingElement("Camera")) {
        bool isLookAt = element->Attribute("type", "lookAt") != nullptr;
        V3 camPos, upDir;
        float nearDist = 0.f, width = 0.f, height = 0.f;
        std::string imageName;
        XmlNode* child = element->FirstChildElement("Position");
        stream.line(child ? child->GetText() : nullptr); stream.get(camPos.x).get(camPos.y).get(camPos.z);
        child = element->FirstChildElement("Up");
        stream.line(child ? child->GetText() : nullptr); stream.get(upDir.x).get(upDir.y).get(upDir.z);
        child = element->FirstChildElement("NearDistance");
        stream.line(child ? child->GetText() : nullptr); stream.get(nearDist);
        child = element->FirstChildElement("ImageResolution");
        stream.line(child ? child->GetText() : nullptr); stream.get(width).get(height);
        child = element->FirstChildElement("ImageName");
        stream.line(child ? child->GetText() : nullptr); stream.get(imageName);
        int iw = (int)width, ih = (int)height;
        V3 gaze, up, right, q;
        float mleft, mright, mbottom, mtop;
        if (isLookAt) {                                 // camera.cpp:25-48
            V3 gazePoint;
            float fovY = 0.f;
            child = element->FirstChildElement("GazePoint");
            if (!child) child = element->FirstChildElement("Gaze");
            stream.line(child ? child->GetText() : nullptr); stream.get(gazePoint.x).get(gazePoint.y).get(gazePoint.z);
            child = element->FirstChildElement("FovY");
            stream.line(child ? child->GetText() : nullptr); stream.get(fovY);
            float aspect = (float)iw / ih;
            mtop = nearDist * std::tan((fovY * (M_PI / 180.0f) / 2.0f));
            mright = mtop * aspect;
            mbottom = -mtop;
            mleft = -mright;
            gaze = makeUnit(gazePoint - camPos);
            V3 tempUp = makeUnit(upDir);
            V3 tempRight = makeUnit(cross(tempUp, gaze));
            up = makeUnit(cross(gaze, tempRight));
        } else {                                        // camera.cpp:5-23
            V3 gazeDir;
            float np[4] = {0, 0, 0, 0};
            child = element->FirstChildElement("Gaze");
            stream.line(child ? child->GetText() : nullptr); stream.get(gazeDir.x).get(gazeDir.y).get(gazeDir.z);
            child = element->FirstChildElement("NearPlane");
            stream.line(child ? child->GetText() : nullptr); stream.get(np[0]).get(np[1]).get(np[2]).get(np[3]);
            mleft = np[0]; mright = np[1]; mbottom = np[2]; mtop = np[3];
            gaze = makeUnit(gazeDir);
            V3 tempUp = makeUnit(upDir);
            float dotvu = dot(tempUp, gaze);             // Camera::GetOrthonormal camera.cpp:50-58
            float relativeSqr = dot(gaze, gaze);
            V3 proj = gaze * (dotvu / relativeSqr);
            up = makeUnit(tempUp - proj);
        }
        // CalculateImagePlaneParams (camera.cpp:60-72)
        V3 middle = camPos + gaze * nearDist;
        V3 w = -gaze;
        right = cross(up, w);
        q = middle + right * mleft + up * mtop;

        cam.position = to_f3(camPos); cam.gaze = to_f3(gaze); cam.up = to_f3(up);
        cam.right = to_f3(right); cam.q = to_f3(q);
        cam.left = mleft; cam.right_ext = mright; cam.bottom = mbottom; cam.top = mtop;
        cam.near_dist = nearDist; cam.width = iw; cam.height = ih;
        std::memset(cam.image_name, 0, sizeof(cam.image_name));
        std::strncpy(cam.image_name, imageName.c_str(), sizeof(cam.image_name) - 1);

        int numSamples = 1;
        child = element->FirstChildElement("NumSamples");
        if (child) { stream.line(child->GetText()); stream.get(numSamples); }
        cam.spp = numSamples;
        float focusDistance = 0.f;
        child = element->FirstChildElement("FocusDistance");
        if (child) { stream.line(child->GetText()); stream.get(focusDistance); }
        cam.focus_distance = focusDistance;
        float apertureSize = 0.f;
        child = element->FirstChildElement("ApertureSize");
        if (child) { stream.line(child->GetText()); stream.get(apertureSize); }
        cam.aperture = apertureSize;

        child = element->FirstChildElement("Renderer");         // parser.cpp:1589-1628
        if (child) {
            std::string rendererType;
            stream.line(child->GetText()); stream.get(rendererType);
            if (rendererType == "PathTracing") {
                child = element->FirstChildElement("RendererParams");
                bool is = false, rr = false, nee = false;
                if (child) {
                    stream.line(child->GetText());
                    std::string param;
                    while (stream.get(param)) {
                        if (param == "NextEventEstimation") nee = true;
                        else if (param == "RussianRoulette") rr = true;
                        else if (param == "ImportanceSampling") is = true;
                    }
                }
                stream.clear();
                cam.path_tracing = 1; cam.importance_sampling = is; cam.next_event = nee; cam.russian_roulette = rr;
            }
        }
        child = element->FirstChildElement("Tonemap");           // parser.cpp:828-869
        if (child) {
            RefStream ts;
            std::string opType = "Photographic";
            XmlNode* c = child->FirstChildElement("TMO");
            if (c) { ts.line(c->GetText()); ts.get(opType); }
            float key = 0.18f, burn = 1.0f, sat = 1.0f, gamma = 2.2f;
            c = child->FirstChildElement("TMOOptions");
            if (c) { ts.line(c->GetText()); ts.get(key).get(burn); }
            c = child->FirstChildElement("Saturation");
            if (c) { ts.line(c->GetText()); ts.get(sat); }
            c = child->FirstChildElement("Gamma");
            if (c) { ts.line(c->GetText()); ts.get(gamma); }
            cam.has_tonemapper = 1; cam.tm_key = key; cam.tm_burn = burn; cam.tm_saturation = sat; cam.tm_gamma = gamma;
        }
        S.cameras.push_back(cam);
    }
}

void Loader::parseLights(XmlNode* root) {             // parser.cpp:984-1107
    XmlNode* lights = root->FirstChildElement("Lights");
    S.ambient = V3(0, 0, 0);
    if (!lights) return;
    RefStream stream;
    XmlNode* child = lights->FirstChildElement("AmbientLight");
    if (child) { stream.line(child->GetText()); stream.get(S.ambient.x).get(S.ambient.y).get(S.ambient.z); }
    for (XmlNode* l = lights->FirstChildElement("PointLight"); l; l = l->NextSiblingElement("PointLight")) {
        int id = 0;
        stream.line(l->Attribute("id")); stream.get(id);
        child = l->FirstChildElement("Position"); stream.line(child ? child->GetText() : nullptr);
        child = l->FirstChildElement("Intensity"); stream.line(child ? child->GetText() : nullptr);
        V3 pos, in;
        stream.get(pos.x).get(pos.y).get(pos.z);
        stream.get(in.x).get(in.y).get(in.z);
        rtg_point_light pl; pl.position = to_f3(pos); pl.intensity = to_f3(in);
        S.point_lights.push_back(pl);
    }
    for (XmlNode* l = lights->FirstChildElement("AreaLight"); l; l = l->NextSiblingElement("AreaLight")) {
        V3 pos, nrm, rad;
        float size = 0.f;
        int id = 0;
        stream.line(l->Attribute("id")); stream.get(id);
        child = l->FirstChildElement("Position"); stream.line(child ? child->GetText() : nullptr); stream.get(pos.x).get(pos.y).get(pos.z);
        child = l->FirstChildElement("Normal"); stream.line(child ? child->GetText() : nullptr); stream.get(nrm.x).get(nrm.y).get(nrm.z);
        child = l->FirstChildElement("Radiance"); stream.line(child ? child->GetText() : nullptr); stream.get(rad.x).get(rad.y).get(rad.z);
        child = l->FirstChildElement("Size"); stream.line(child ? child->GetText() : nullptr); stream.get(size);
        rtg_area_light al;                                 // areaLight.h:18-31
        al.position = to_f3(pos); al.normal = to_f3(nrm); al.radiance = to_f3(rad);
        al.extent = size; al.area = size * size;
        V3 u, v;
        orthonormalBasis(nrm, u, v);
        al.u = to_f3(u); al.v = to_f3(v);
        S.area_lights.push_back(al);
    }
    for (XmlNode* l = lights->FirstChildElement("DirectionalLight"); l; l = l->NextSiblingElement("DirectionalLight")) {
        V3 rad, dir;
        int id = 0;
        stream.line(l->Attribute("id")); stream.get(id);
        child = l->FirstChildElement("Direction"); stream.line(child ? child->GetText() : nullptr); stream.get(dir.x).get(dir.y).get(dir.z);
        child = l->FirstChildElement("Radiance"); stream.line(child ? child->GetText() : nullptr); stream.get(rad.x).get(rad.y).get(rad.z);
        rtg_directional_light dl; dl.dir = to_f3(makeUnit(dir)); dl.radiance = to_f3(rad);   // directionalLight.h:15-20
        S.dir_lights.push_back(dl);
    }
    for (XmlNode* l = lights->FirstChildElement("SpotLight"); l; l = l->NextSiblingElement("SpotLight")) {
        V3 pos, dir, in;
        int id = 0;
        float cov = 0.f, fall = 0.f;
        stream.line(l->Attribute("id")); stream.get(id);
        child = l->FirstChildElement("Position"); stream.line(child ? child->GetText() : nullptr); stream.get(pos.x).get(pos.y).get(pos.z);
        child = l->FirstChildElement("Direction"); stream.line(child ? child->GetText() : nullptr); stream.get(dir.x).get(dir.y).get(dir.z);
        child = l->FirstChildElement("Intensity"); stream.line(child ? child->GetText() : nullptr); stream.get(in.x).get(in.y).get(in.z);
        child = l->FirstChildElement("CoverageAngle"); stream.line(child ? child->GetText() : nullptr); stream.get(cov);
        child = l->FirstChildElement("FalloffAngle"); stream.line(child ? child->GetText() : nullptr); stream.get(fall);
        rtg_spot_light sl;                                 // spotLight.h:17-26
        sl.position = to_f3(pos); sl.dir = to_f3(makeUnit(dir)); sl.intensity = to_f3(in);
        sl.coverage_deg = cov; sl.falloff_deg = fall;
        const double DEG2RAD = (M_PI / 180.0f);
        sl.cos_half_coverage = std::cos((cov * DEG2RAD / 2.0f));
        sl.cos_half_falloff = std::cos((fall * DEG2RAD / 2.0f));
        S.spot_lights.push_back(sl);
    }
}

void Loader::parseBRDFs(XmlNode* root) {              // parser.cpp:870-982
    XmlNode* b = root->FirstChildElement("BRDFs");
    if (!b) return;
    RefStream stream;
    struct Kind { const char* tag; int type; const char* flag; };
    const Kind kinds[] = {
        {"ModifiedBlinnPhong", RTG_BRDF_MODIFIED_BLINN_PHONG, "normalized"},
        {"OriginalBlinnPhong", RTG_BRDF_BLINN_PHONG, nullptr},
        {"OriginalPhong", RTG_BRDF_PHONG, nullptr},
        {"ModifiedPhong", RTG_BRDF_MODIFIED_PHONG, "normalized"},
        {"TorranceSparrow", RTG_BRDF_TORRANCE_SPARROW, "kdfresnel"},
    };
    for (const Kind& k : kinds) {
        for (XmlNode* e = b->FirstChildElement(k.tag); e; e = e->NextSiblingElement(k.tag)) {
            rtg_brdf br;
            std::memset(&br, 0, sizeof(br));
            int id = -1;
            stream.line(e->Attribute("id")); stream.get(id);
            bool flag = k.flag && e->Attribute(k.flag, "true") != nullptr;
            float exponent = 0.f;
            XmlNode* ex = e->FirstChildElement("Exponent");
            stream.line(ex ? ex->GetText() : nullptr); stream.get(exponent);
            br.id = id; br.type = k.type; br.exponent = exponent;
            if (k.type == RTG_BRDF_TORRANCE_SPARROW) { br.energy_conserving = 1; br.kd_fresnel = flag; }
            else br.energy_conserving = flag;
            S.brdfs.push_back(br);
        }
    }
}

void Loader::parseMaterials(XmlNode* root) {          // parser.cpp:1109-1278
    XmlNode* mats = root->FirstChildElement("Materials");
    if (!mats) fail(RTG_ERR_PARSE, "missing <Materials>");
    RefStream stream;
    rtg_material m;                                     // ONE object, reused
    std::memset(&m, 0, sizeof(m));
    m.brdf = -1;
    for (XmlNode* e = mats->FirstChildElement("Material"); e; e = e->NextSiblingElement("Material")) {
        stream.line(e->Attribute("id")); stream.get(m.id);
        if (e->Attribute("BRDF")) {
            int brdfID = -1;
            stream.line(e->Attribute("BRDF")); stream.get(brdfID);
            int found = -1;
            for (size_t i = 0; i < S.brdfs.size(); ++i) if (S.brdfs[i].id == brdfID) { found = (int)i; break; }
            m.brdf = found;
        }
        if (e->Attribute("type", "mirror")) m.type = RTG_MAT_MIRROR;
        else if (e->Attribute("type", "dielectric")) m.type = RTG_MAT_DIELECTRIC;
        else if (e->Attribute("type", "conductor")) m.type = RTG_MAT_CONDUCTOR;
        else m.type = RTG_MAT_DEFAULT;
        bool degamma = e->Attribute("degamma", "true") != nullptr;
        const float gamma = 2.2f;
        auto read3 = [&](XmlNode* c, rtg_float3& v) {
            stream.line(c->GetText());
            stream.get(v.x).get(v.y).get(v.z);
            if (degamma) { v.x = std::pow(v.x, gamma); v.y = std::pow(v.y, gamma); v.z = std::pow(v.z, gamma); }
        };
        XmlNode* c = e->FirstChildElement("AmbientReflectance");
        if (c) read3(c, m.ambient);
        c = e->FirstChildElement("DiffuseReflectance");
        if (c) read3(c, m.diffuse);
        c = e->FirstChildElement("SpecularReflectance");
        if (c) read3(c, m.specular);
        c = e->FirstChildElement("MirrorReflectance");
        if (c) read3(c, m.mirror); else m.mirror = rtg_float3{0.f, 0.f, 0.f};
        c = e->FirstChildElement("RefractionIndex");
        if (c) { stream.line(c->GetText()); stream.get(m.refractive_index); } else m.refractive_index = 1.0f;
        c = e->FirstChildElement("AbsorptionCoefficient");
        if (c) { stream.line(c->GetText()); stream.get(m.absorption.x).get(m.absorption.y).get(m.absorption.z); }
        else m.absorption = rtg_float3{0.f, 0.f, 0.f};
        c = e->FirstChildElement("AbsorptionIndex");
        if (c) { stream.line(c->GetText()); stream.get(m.absorption_index); } else m.absorption_index = 0.0f;
        c = e->FirstChildElement("PhongExponent");
        if (c) { stream.line(c->GetText()); stream.get(m.phong_exponent); } else m.phong_exponent = 1.0f;
        c = e->FirstChildElement("Roughness");
        if (c) { stream.line(c->GetText()); stream.get(m.roughness); } else m.roughness = 0.0f;
        S.materials.push_back(m);
    }
}

void Loader::parseTextures(XmlNode* root, RefStream& stream) {   // parser.cpp:84-228
    XmlNode* element = root->FirstChildElement("Textures");
    if (!element) return;
    XmlNode* images = element->FirstChildElement("Images");
    if (images) {
        for (XmlNode* im = images->FirstChildElement("Image"); im; im = im->NextSiblingElement("Image")) {
            int id = 0;
            std::string filename;
            stream.line(im->Attribute("id")); stream.get(id);
            stream.line(im->GetText()); stream.get(filename);
            HostScene::ImageStore st;
            std::string err;
            if (filename.find(".exr") != std::string::npos) {          // HDRImage (parser.cpp:103-107)
                if (!load_exr("inputs/" + filename, st.width, st.height, st.texels, err))
                    fail(err.find("not supported") != std::string::npos ? RTG_ERR_UNSUPPORTED : RTG_ERR_IO, err);
                st.channels = 3;
                st.is_hdr = 1;
            } else {                                                    // LDRImage (parser.cpp:110)
                Image8 img;
                if (!load_image8("inputs/" + filename, img, err))
                    fail(err.rfind("unsupported", 0) == 0 ? RTG_ERR_UNSUPPORTED : RTG_ERR_IO, err);
                st.width = img.width; st.height = img.height; st.channels = img.channels;
                st.texels.assign(img.data.begin(), img.data.end());
            }
            st.id = id;
            S.imageStore.push_back(std::move(st));
            imageIds.push_back(id);
        }
    }
    for (XmlNode* tm = element->FirstChildElement("TextureMap"); tm; tm = tm->NextSiblingElement("TextureMap")) {
        int textureId = 0;
        std::string textureType, decalMode;
        stream.line(tm->Attribute("id")); stream.get(textureId);
        stream.line(tm->Attribute("type")); stream.get(textureType);
        XmlNode* child = tm->FirstChildElement("DecalMode");
        stream.line(child ? child->GetText() : nullptr); stream.get(decalMode);
        TexRec tr;
        std::memset(&tr.t, 0, sizeof(tr.t));
        tr.t.id = textureId;
        tr.decal = decalMode;
        // Texture::SetTextureType / SetOperationMode (texture.h:66-98)
        if (decalMode == "replace_kd" || decalMode == "blend_kd") tr.t.slot = RTG_TEXSLOT_DIFFUSE;
        else if (decalMode == "replace_ks") tr.t.slot = RTG_TEXSLOT_SPECULAR;
        else if (decalMode == "replace_normal") tr.t.slot = RTG_TEXSLOT_NORMAL;
        else if (decalMode == "bump_normal") tr.t.slot = RTG_TEXSLOT_BUMP;
        else if (decalMode == "replace_all") tr.t.slot = RTG_TEXSLOT_REPLACE_ALL;
        else tr.t.slot = RTG_TEXSLOT_NONE;
        tr.t.blend = decalMode == "blend_kd";
        tr.t.is_background = decalMode == "replace_background";
        tr.t.image = -1;
        if (textureType == "image") {
            int imageId = 0;
            child = tm->FirstChildElement("ImageId");
            stream.line(child ? child->GetText() : nullptr); stream.get(imageId);
            std::string interp = "nearest";
            child = tm->FirstChildElement("Interpolation");
            if (child) { stream.line(child->GetText()); stream.get(interp); }
            float normalizer = 255.0f, mult = 1.0f;
            child = tm->FirstChildElement("Normalizer");
            if (child) { stream.line(child->GetText()); stream.get(normalizer); }
            child = tm->FirstChildElement("BumpFactor");
            if (child) { stream.line(child->GetText()); stream.get(mult); }
            int img = -1;
            for (size_t i = 0; i < imageIds.size(); ++i) if (imageIds[i] == imageId) { img = (int)i; break; }
            if (img < 0) fail(RTG_ERR_PARSE, "TextureMap: no image with id " + std::to_string(imageId));
            tr.t.kind = RTG_TEX_IMAGE;
            tr.t.image = img;
            tr.t.nearest = interp == "nearest";
            tr.t.normalizer = normalizer;
            tr.t.bump_factor = mult;
        } else if (textureType == "perlin") {
            std::string conv = "linear";
            child = tm->FirstChildElement("NoiseConversion");
            if (child) { stream.line(child->GetText()); stream.get(conv); }
            float scale = 1.0f, bump = 1.0f;
            child = tm->FirstChildElement("NoiseScale");
            if (child) { stream.line(child->GetText()); stream.get(scale); }
            child = tm->FirstChildElement("BumpFactor");
            if (child) { stream.line(child->GetText()); stream.get(bump); }
            tr.t.kind = RTG_TEX_PERLIN;
            tr.t.noise_scale = scale;
            tr.t.noise_abs = conv == "absval";
            tr.t.bump_factor = bump;
            tr.t.normalizer = 1.0f;
        } else {
            continue;   // "checkerboard" is unimplemented in the reference too (parser.cpp:220-224)
        }
        if (tr.t.is_background) S.bgTexture = (int)texs.size();
        texs.push_back(tr);
    }
}

void Loader::setupTextures(int* tex, std::string ids) {   // parser.cpp:612-650
    size_t last = 0, next = 0;
    while ((next = ids.find(" ", last)) != std::string::npos) {
        std::string idStr = ids.substr(last, next - last);
        int id;
        try { id = std::stoi(idStr); } catch (...) { fail(RTG_ERR_PARSE, "bad texture id '" + idStr + "'"); }
        int found = -1;
        for (size_t i = 0; i < texs.size(); ++i) if (texs[i].t.id == id) { found = (int)i; break; }
        if (found < 0) break;
        switch (texs[found].t.slot) {
            case RTG_TEXSLOT_DIFFUSE: tex[0] = found; break;
            case RTG_TEXSLOT_SPECULAR: tex[1] = found; break;
            case RTG_TEXSLOT_NORMAL: tex[2] = found; break;
            case RTG_TEXSLOT_BUMP: tex[3] = found; break;
            case RTG_TEXSLOT_REPLACE_ALL: tex[4] = found; break;
            default: break;
        }
        last = next + 1;
    }
}

void Loader::computeTransform(Xform& xf, const std::string& str) {   // parser.cpp:651-723
    size_t idx = 0;
    std::vector<M4> inv;
    auto digit = [&](size_t i) -> int {
        if (i >= str.size()) fail(RTG_ERR_PARSE, "truncated transformation list '" + str + "'");
        return int(str[i] - '0');
    };
    while (str.size() >= 1 && idx < str.size() - 1) {
        if (str[idx] == 'r') {
            int id = digit(idx + 1);
            if (id < 1 || id > (int)rotations.size()) fail(RTG_ERR_PARSE, "rotation id out of range");
            Rot r = rotations[id - 1];
            float angle = r.w * (M_PI / 180.0f);   // float, as parser.cpp:665
            M4 rot, invRot;
            rot.valid = invRot.valid = false;
            if (r.x >= 0.99 && r.y <= 0.001 && r.z <= 0.0001) { rot = M4::rotX(angle); invRot = M4::rotX(-angle); }
            if (r.y >= 0.99 && r.x <= 0.001 && r.z <= 0.0001) { rot = M4::rotY(angle); invRot = M4::rotY(-angle); }
            if (r.z >= 0.99 && r.x <= 0.001 && r.y <= 0.0001) { rot = M4::rotZ(angle); invRot = M4::rotZ(-angle); }
            if (!rot.valid) fail(RTG_ERR_UNSUPPORTED, "rotation about a non-principal axis (the reference leaves a 0x0 matrix)");
            inv.push_back(invRot);
            xf.transform = rot * xf.transform;
        } else if (str[idx] == 't') {
            int id = digit(idx + 1);
            if (id < 1 || id > (int)translations.size()) fail(RTG_ERR_PARSE, "translation id out of range");
            V3 t = translations[id - 1];
            inv.push_back(M4::translation(-t.x, -t.y, -t.z));
            xf.transform = M4::translation(t.x, t.y, t.z) * xf.transform;
        } else if (str[idx] == 's') {
            int id = digit(idx + 1);
            if (id < 1 || id > (int)scalings.size()) fail(RTG_ERR_PARSE, "scaling id out of range");
            V3 s = scalings[id - 1];
            inv.push_back(M4::scale(1.0f / s.x, 1.0f / s.y, 1.0f / s.z));
            xf.transform = M4::scale(s.x, s.y, s.z) * xf.transform;
        }
        idx += 3;
    }
    xf.inverse = M4::identity();
    for (const M4& m : inv) xf.inverse = xf.inverse * m;
    xf.invTranspose = xf.inverse.transpose();
}

void Loader::computeFaceProperties(FaceRec& f, Geometry& g) {   // parser.cpp:579-747
    const V3 a = g.vertex(f.v0), b = g.vertex(f.v1), c = g.vertex(f.v2);
    f.center = (a + b + c) / 3.0f;
    f.n = makeUnit(cross(b - a, c - a));
    f.bbox.mn = V3(std::min(std::min(a.x, b.x), c.x), std::min(std::min(a.y, b.y), c.y), std::min(std::min(a.z, b.z), c.z));
    f.bbox.mx = V3(std::max(std::max(a.x, b.x), c.x), std::max(std::max(a.y, b.y), c.y), std::max(std::max(a.z, b.z), c.z));
    double e1 = len(a - b), e2 = len(a - c), e3 = len(b - c);
    double s = (e1 + e2 + e3) / 2.0f;
    f.area = std::sqrt(s * (s - e1) * (s - e2) * (s - e3));
    g.surfaceArea += f.area;
}

BBox Loader::transformBoundingBox(const BBox& o, const M4& t) {   // parser.cpp:749-805
    BBox r;
    r.mx = V3(-INFINITY, -INFINITY, -INFINITY);
    r.mn = V3(INFINITY, INFINITY, INFINITY);
    std::vector<V3> corners;
    corners.push_back(o.mx);
    corners.push_back(o.mn);
    V3 ext = o.mx - o.mn;
    V3 c = o.mx; c.x -= ext.x; corners.push_back(c);
    c = o.mx; c.y -= ext.y; corners.push_back(c);
    c = o.mx; c.z -= ext.z; corners.push_back(c);
    c = o.mx; c.x -= ext.x; c.y -= ext.y; corners.push_back(c);
    c = o.mx; c.x -= ext.x; c.z -= ext.z; corners.push_back(c);
    c = o.mx; c.y -= ext.y; c.z -= ext.z; corners.push_back(c);
    for (V3& k : corners) {
        k = applyPoint(t, k);
        r.mx.x = std::max(k.x, r.mx.x); r.mx.y = std::max(k.y, r.mx.y); r.mx.z = std::max(k.z, r.mx.z);
        r.mn.x = std::min(k.x, r.mn.x); r.mn.y = std::min(k.y, r.mn.y); r.mn.z = std::min(k.z, r.mn.z);
    }
    return r;
}

void Loader::parseMeshes(XmlNode* root, const char* elemName) {   // parser.cpp:1280-1496
    XmlNode* objects = root->FirstChildElement("Objects");
    if (!objects) fail(RTG_ERR_PARSE, "missing <Objects>");
    RefStream stream;
    const bool isLight = std::strcmp(elemName, "LightMesh") == 0;
    for (XmlNode* element = objects->FirstChildElement(elemName); element;
         element = element->NextSiblingElement(elemName)) {
        XmlNode* child = element->FirstChildElement("Faces");
        if (!child) fail(RTG_ERR_PARSE, "mesh without <Faces>");
        bool hasPly = child->Attribute("plyFile") != nullptr;
        Geometry g;
        ShapeRec sh;
        sh.lightMesh = isLight;
        V3 radiance(0, 0, 0);
        if (isLight) {
            child = element->FirstChildElement("Radiance");
            if (child) { stream.line(child->GetText()); stream.get(radiance.x).get(radiance.y).get(radiance.z); }
        }
        if (!hasPly) { g.verts = vertex_data; g.uv = texCoords; }
        stream.line(element->Attribute("id")); stream.get(sh.id);
        child = element->FirstChildElement("Textures");
        if (child) setupTextures(sh.tex, need_text(child, "Textures") + " ");
        child = element->FirstChildElement("Transformations");
        sh.xf.transform = M4::identity();
        sh.xf.inverse = M4::identity();
        sh.xf.invTranspose = M4::identity();
        if (child) computeTransform(sh.xf, need_text(child, "Transformations"));
        child = element->FirstChildElement("Material");
        stream.line(child ? child->GetText() : nullptr);
        int matId = 0;
        stream.get(matId);
        sh.material = matId;
        child = element->FirstChildElement("MotionBlur");
        if (child) {
            stream.line(child->GetText());
            stream.get(sh.mbv.x).get(sh.mbv.y).get(sh.mbv.z);
            sh.motionBlur = true;
            S.motionBlurEnabled = true;
        }
        child = element->FirstChildElement("Faces");
        if (child->Attribute("vertexOffset")) { stream.line(child->Attribute("vertexOffset")); stream.get(g.vertexOffset); }
        if (child->Attribute("textureOffset")) { stream.line(child->Attribute("textureOffset")); stream.get(g.textureOffset); }

        BBox bbox;
        bbox.mx = V3(std::numeric_limits<float>::min(), std::numeric_limits<float>::min(), std::numeric_limits<float>::min());
        bbox.mn = V3(std::numeric_limits<float>::max(), std::numeric_limits<float>::max(), std::numeric_limits<float>::max());
        auto grow = [&](const FaceRec& f) {           // Scene::updateBBox (parser.cpp:817-827)
            bbox.mn.x = std::min(f.bbox.mn.x, bbox.mn.x); bbox.mn.y = std::min(f.bbox.mn.y, bbox.mn.y);
            bbox.mn.z = std::min(f.bbox.mn.z, bbox.mn.z);
            bbox.mx.x = std::max(f.bbox.mx.x, bbox.mx.x); bbox.mx.y = std::max(f.bbox.mx.y, bbox.mx.y);
            bbox.mx.z = std::max(f.bbox.mx.z, bbox.mx.z);
        };
        if (hasPly) {
            std::string filename;
            stream.put(child->Attribute("plyFile")); stream.get(filename);
            PlyData ply;
            std::string err;
            if (!load_ply(child->Attribute("plyFile"), ply, err)) fail(RTG_ERR_IO, err);
            for (auto& p : ply.positions) g.verts.push_back(V3((float)p[0], (float)p[1], (float)p[2]));
            for (auto& fi : ply.faces) {
                if (fi.size() == 3) {
                    FaceRec f; f.v0 = fi[0] + 1; f.v1 = fi[1] + 1; f.v2 = fi[2] + 1;
                    computeFaceProperties(f, g); grow(f); g.faces.push_back(f);
                } else if (fi.size() == 4) {
                    FaceRec f1; f1.v0 = fi[0] + 1; f1.v1 = fi[1] + 1; f1.v2 = fi[2] + 1;
                    computeFaceProperties(f1, g); grow(f1); g.faces.push_back(f1);
                    FaceRec f2; f2.v0 = fi[2] + 1; f2.v1 = fi[3] + 1; f2.v2 = fi[0] + 1;
                    computeFaceProperties(f2, g); grow(f2); g.faces.push_back(f2);
                }
            }
        } else {
            stream.line(child->GetText());
            FaceRec f;
            while (!stream.get(f.v0).eof()) {
                stream.get(f.v1).get(f.v2);
                if (stream.fail()) fail(RTG_ERR_PARSE, "malformed <Faces>");
                computeFaceProperties(f, g);
                grow(f);
                g.faces.push_back(f);
            }
        }
        stream.clear();
        if (g.faces.empty()) fail(RTG_ERR_PARSE, "mesh without faces (the reference's BVH build cannot handle it)");
        g.bbox = bbox;
        sh.geometry = (int)geos.size();
        geos.push_back(std::move(g));
        if (isLight) {
            if (sh.material < 1 || sh.material > (int)S.materials.size()) fail(RTG_ERR_PARSE, "LightMesh material out of range");
            rtg_material& mat = S.materials[sh.material - 1];   // parser.cpp:1484-1487
            mat.type = RTG_MAT_EMISSIVE;
            mat.radiance = to_f3(radiance);
            rtg_mesh_light ml;
            ml.object = (int32_t)shapes.size();     // objects[] follow scene.meshes order
            ml.radiance = to_f3(radiance);
            S.mesh_lights.push_back(ml);
        }
        shapes.push_back(sh);
    }
}

// Mesh::ConstructBVH / RecursiveBVHBuild / RecomputeBoundingBox (mesh.cpp:23-156).
void Loader::constructBVH(Geometry& g, std::vector<rtg_bvh_node>& out) {
    const int n = (int)g.faces.size();
    struct Node { BBox bbox; int left = -1; uint32_t first = 0, count = 0; };
    std::vector<Node> nodes(size_t(2) * n - 1);
    nodes[0].bbox = g.bbox;
    nodes[0].first = 0;
    nodes[0].count = (uint32_t)n;
    int nextFree = 1;
    std::vector<int> todo{0};
    while (!todo.empty()) {
        int idx = todo.back();
        todo.pop_back();
        Node& node = nodes[idx];
        if (node.count < 2) continue;
        float lenX = node.bbox.mx.x - node.bbox.mn.x;
        float lenY = node.bbox.mx.y - node.bbox.mn.y;
        float lenZ = node.bbox.mx.z - node.bbox.mn.z;
        float split;
        int axis;
        if (lenX > lenY) {
            if (lenX > lenZ) { split = node.bbox.mn.x + lenX * 0.5f; axis = 0; }
            else { split = node.bbox.mn.z + lenZ * 0.5f; axis = 2; }
        } else {
            if (lenY > lenZ) { split = node.bbox.mn.y + lenY * 0.5f; axis = 1; }
            else { split = node.bbox.mn.z + lenZ * 0.5f; axis = 2; }
        }
        int i = (int)node.first;
        int j = i + (int)node.count - 1;
        while (i <= j) {
            if (g.faces[i].center[axis] < split) i++;
            else { std::swap(g.faces[i], g.faces[j]); j--; }
        }
        int leftCount = i - (int)node.first;
        if (leftCount == 0 || leftCount == (int)node.count) continue;
        int li = nextFree++, ri = nextFree++;
        nodes[li].first = node.first; nodes[li].count = leftCount;
        nodes[ri].first = i; nodes[ri].count = node.count - leftCount;
        node.left = li;
        node.count = 0;
        for (int k : {li, ri}) {
            Node& c = nodes[k];
            c.bbox.mn = V3(INFINITY, INFINITY, INFINITY);
            c.bbox.mx = V3(-INFINITY, -INFINITY, -INFINITY);
            for (uint32_t f = 0; f < c.count; ++f) {
                const FaceRec& fr = g.faces[c.first + f];
                c.bbox.mn.x = std::min(c.bbox.mn.x, fr.bbox.mn.x); c.bbox.mn.y = std::min(c.bbox.mn.y, fr.bbox.mn.y);
                c.bbox.mn.z = std::min(c.bbox.mn.z, fr.bbox.mn.z);
                c.bbox.mx.x = std::max(c.bbox.mx.x, fr.bbox.mx.x); c.bbox.mx.y = std::max(c.bbox.mx.y, fr.bbox.mx.y);
                c.bbox.mx.z = std::max(c.bbox.mx.z, fr.bbox.mx.z);
            }
        }
        // recursion order: left subtree completely, then right (pre-order allocation)
        todo.push_back(ri);
        todo.push_back(li);
    }
    out.resize(nextFree);
    for (int k = 0; k < nextFree; ++k) {
        rtg_bvh_node& o = out[k];
        const Node& s = nodes[k];
        o.bmin[0] = s.bbox.mn.x; o.bmin[1] = s.bbox.mn.y; o.bmin[2] = s.bbox.mn.z;
        o.bmax[0] = s.bbox.mx.x; o.bmax[1] = s.bbox.mx.y; o.bmax[2] = s.bbox.mx.z;
        o.left = s.left;
        o.first = (int32_t)s.first;
        o.count = s.left >= 0 ? 0 : (int32_t)s.count;
        o.pad0 = 0;
    }
}

void Loader::flatten() {
    // geometry: faces + BVH
    std::vector<int> geoMesh(geos.size(), -1);
    for (size_t gi = 0; gi < geos.size(); ++gi) {
        Geometry& g = geos[gi];
        std::vector<rtg_bvh_node> nodes;
        const auto tb = std::chrono::steady_clock::now();
        if (!S.deferBvh) constructBVH(g, nodes);
        bvhSeconds += std::chrono::duration<double>(std::chrono::steady_clock::now() - tb).count();
        rtg_mesh m;
        std::memset(&m, 0, sizeof(m));
        m.face_offset = (int32_t)S.faces.size();
        m.face_count = (int32_t)g.faces.size();
        m.node_offset = (int32_t)S.nodes.size();
        m.node_count = (int32_t)nodes.size();
        m.has_uv = g.uv.empty() ? 0 : 1;
        m.surface_area = g.surfaceArea;
        for (const FaceRec& f : g.faces) {
            rtg_face o;
            std::memset(&o, 0, sizeof(o));
            o.v0 = to_f3(g.vertex(f.v0)); o.v1 = to_f3(g.vertex(f.v1)); o.v2 = to_f3(g.vertex(f.v2));
            o.n = to_f3(f.n);
            if (m.has_uv) {
                auto a = g.texcoord(f.v0), b = g.texcoord(f.v1), c = g.texcoord(f.v2);
                o.uv0[0] = a[0]; o.uv0[1] = a[1]; o.uv1[0] = b[0]; o.uv1[1] = b[1]; o.uv2[0] = c[0]; o.uv2[1] = c[1];
            }
            o.area = f.area;
            S.faces.push_back(o);
        }
        S.nodes.insert(S.nodes.end(), nodes.begin(), nodes.end());
        geoMesh[gi] = (int)S.meshes.size();
        S.meshes.push_back(m);
    }
    auto check_mat = [&](int m) {
        if (m < 1 || m > (int)S.materials.size()) fail(RTG_ERR_PARSE, "material id " + std::to_string(m) + " out of range");
    };
    // objects: scene.meshes order, then spheres
    for (const ShapeRec& sh : shapes) {
        rtg_object o;
        std::memset(&o, 0, sizeof(o));
        o.kind = sh.isInstance ? RTG_OBJ_INSTANCE : RTG_OBJ_MESH;
        check_mat(sh.material);
        o.material = sh.material - 1;
        o.mesh = geoMesh[sh.geometry];
        o.id = sh.id;
        if (S.materials[o.material].type == RTG_MAT_EMISSIVE) o.flags |= RTG_OBJF_SHADOW_SKIP;
        if (!S.meshes[o.mesh].has_uv) o.flags |= RTG_OBJF_NORMAL_TWICE;
        if (sh.motionBlur) o.flags |= RTG_OBJF_MOTION_BLUR;
        o.tex_diffuse = sh.tex[0]; o.tex_specular = sh.tex[1]; o.tex_replace_all = sh.tex[4];
        // normal / bump maps are read by IntersectFace of the BASE mesh (mesh.cpp:263-358,
        // `this` is the base Mesh for an instance): an instance takes its base mesh's maps
        const ShapeRec& geoOwner = sh.isInstance ? shapes[sh.parentShape] : sh;
        o.tex_normal = geoOwner.tex[2];
        o.tex_bump = geoOwner.tex[3];
        sh.xf.inverse.to(o.inv_transform);
        sh.xf.invTranspose.to(o.inv_transpose);
        sh.xf.transform.to(o.transform);
        if (sh.isInstance) {
            shapes[sh.parentShape].xf.invTranspose.to(o.base_inv_transpose);
            o.bbox_min[0] = sh.bbox.mn.x; o.bbox_min[1] = sh.bbox.mn.y; o.bbox_min[2] = sh.bbox.mn.z;
            o.bbox_max[0] = sh.bbox.mx.x; o.bbox_max[1] = sh.bbox.mx.y; o.bbox_max[2] = sh.bbox.mx.z;
        } else {
            sh.xf.invTranspose.to(o.base_inv_transpose);
            const BBox& b = geos[sh.geometry].bbox;
            o.bbox_min[0] = b.mn.x; o.bbox_min[1] = b.mn.y; o.bbox_min[2] = b.mn.z;
            o.bbox_max[0] = b.mx.x; o.bbox_max[1] = b.mx.y; o.bbox_max[2] = b.mx.z;
        }
        o.motion_blur = to_f3(sh.mbv);
        o.radius = 0.f;
        S.objects.push_back(o);
    }
    for (const SphereRec& sp : spheres) {
        rtg_object o;
        std::memset(&o, 0, sizeof(o));
        o.kind = RTG_OBJ_SPHERE;
        check_mat(sp.material);
        o.material = sp.material - 1;
        o.mesh = -1;
        if (sp.motionBlur) o.flags |= RTG_OBJF_MOTION_BLUR;   // spheres are never skipped by shadow rays
        o.tex_diffuse = sp.tex[0]; o.tex_specular = sp.tex[1]; o.tex_normal = sp.tex[2];
        o.tex_bump = sp.tex[3]; o.tex_replace_all = sp.tex[4];
        sp.xf.inverse.to(o.inv_transform);
        sp.xf.invTranspose.to(o.inv_transpose);
        sp.xf.invTranspose.to(o.base_inv_transpose);
        sp.xf.transform.to(o.transform);
        if (sp.centerId < 1 || sp.centerId > (int)vertex_data.size()) fail(RTG_ERR_PARSE, "sphere center id out of range");
        o.center = to_f3(vertex_data[sp.centerId - 1]);
        o.radius = sp.radius;
        o.motion_blur = to_f3(sp.mbv);
        S.objects.push_back(o);
    }
    for (const TexRec& t : texs) S.textures.push_back(t.t);
}

}  // namespace

// ---------------------------------------------------------------------------
int HostScene::load(const std::string& path, std::string& err) {
    try {
        Loader L(*this);
        L.load(path);
    } catch (const LoadError& e) {
        err = e.what();
        return e.code;
    } catch (const std::exception& e) {
        err = e.what();
        return RTG_ERR_PARSE;
    }
    finalize();
    return RTG_OK;
}

void HostScene::finalize() {
    images.clear();
    for (auto& st : imageStore) {
        rtg_image im;
        std::memset(&im, 0, sizeof(im));
        im.id = st.id; im.width = st.width; im.height = st.height; im.channels = st.channels;
        im.is_hdr = st.is_hdr;
        im.texels = st.texels.data();
        images.push_back(im);
    }
    std::memset(&desc, 0, sizeof(desc));
    std::memcpy(desc.background, background, sizeof(background));
    desc.shadow_epsilon = shadowEps;
    desc.max_recursion_depth = maxDepth;
    desc.bg_texture = bgTexture;
    desc.ambient_light = to_f3(ambient);
    desc.cameras = cameras.data(); desc.num_cameras = (int32_t)cameras.size();
    desc.materials = materials.data(); desc.num_materials = (int32_t)materials.size();
    desc.brdfs = brdfs.data(); desc.num_brdfs = (int32_t)brdfs.size();
    desc.point_lights = point_lights.data(); desc.num_point_lights = (int32_t)point_lights.size();
    desc.area_lights = area_lights.data(); desc.num_area_lights = (int32_t)area_lights.size();
    desc.dir_lights = dir_lights.data(); desc.num_dir_lights = (int32_t)dir_lights.size();
    desc.spot_lights = spot_lights.data(); desc.num_spot_lights = (int32_t)spot_lights.size();
    desc.env_lights = env_lights.data(); desc.num_env_lights = (int32_t)env_lights.size();
    desc.textures = textures.data(); desc.num_textures = (int32_t)textures.size();
    desc.images = images.data(); desc.num_images = (int32_t)images.size();
    desc.objects = objects.data(); desc.num_objects = (int32_t)objects.size();
    desc.meshes = meshes.data(); desc.num_meshes = (int32_t)meshes.size();
    desc.faces = faces.data(); desc.num_faces = (int64_t)faces.size();
    desc.nodes = nodes.data(); desc.num_nodes = (int64_t)nodes.size();
    desc.mesh_lights = mesh_lights.data(); desc.num_mesh_lights = (int32_t)mesh_lights.size();
}

}  // namespace rtg
