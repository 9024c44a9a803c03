// Asset readers for the scene loader: PLY meshes (replaces happly, parser.cpp:1396-1444), LDR
// images (PNG / PNM; replaces stb_image as used by LDRImage.h:37-44) and OpenEXR images (replaces
// tinyexr as used by HDRImage.h:45-72: the reference's only HDR image path, environment maps
// included).  JPEG is refused with RTG_ERR_UNSUPPORTED (a parity gap; a front end
// over the reference's own loaders -- integration/dorkrt -- may still hand decoded texels to
// rtg_scene_create).
#include "host_assets.hpp"

#include <zlib.h>

#include <cmath>
#include <cstdint>
#include <cstring>
#include <fstream>
#include <sstream>
#include <algorithm>

namespace rtg {

static bool read_file(const std::string& path, std::string& out) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    std::stringstream ss;
    ss << f.rdbuf();
    out = ss.str();
    return true;
}

// ============================================================================
// PLY (ascii / binary little / big endian); vertex x,y,z and a face index list
// named vertex_indices or vertex_index, as happly::PLYData::getVertexPositions /
// getFaceIndices read them.
// ============================================================================
namespace {
enum PType { P_I8, P_U8, P_I16, P_U16, P_I32, P_U32, P_F32, P_F64, P_BAD };
PType ptype(const std::string& t) {
    if (t == "char" || t == "int8") return P_I8;
    if (t == "uchar" || t == "uint8") return P_U8;
    if (t == "short" || t == "int16") return P_I16;
    if (t == "ushort" || t == "uint16") return P_U16;
    if (t == "int" || t == "int32") return P_I32;
    if (t == "uint" || t == "uint32") return P_U32;
    if (t == "float" || t == "float32") return P_F32;
    if (t == "double" || t == "float64") return P_F64;
    return P_BAD;
}
int psize(PType t) {
    switch (t) {
        case P_I8: case P_U8: return 1;
        case P_I16: case P_U16: return 2;
        case P_I32: case P_U32: case P_F32: return 4;
        case P_F64: return 8;
        default: return 0;
    }
}
struct PProp { std::string name; bool list = false; PType count = P_BAD, type = P_BAD; };
struct PElem { std::string name; size_t count = 0; std::vector<PProp> props; };

struct BinReader {
    const unsigned char* p; const unsigned char* end; bool swap;
    bool ok = true;
    double read(PType t) {
        int n = psize(t);
        if (p + n > end) { ok = false; return 0; }
        unsigned char b[8];
        for (int i = 0; i < n; ++i) b[i] = swap ? p[n - 1 - i] : p[i];
        p += n;
        switch (t) {
            case P_I8: { int8_t v; std::memcpy(&v, b, 1); return v; }
            case P_U8: { uint8_t v; std::memcpy(&v, b, 1); return v; }
            case P_I16: { int16_t v; std::memcpy(&v, b, 2); return v; }
            case P_U16: { uint16_t v; std::memcpy(&v, b, 2); return v; }
            case P_I32: { int32_t v; std::memcpy(&v, b, 4); return v; }
            case P_U32: { uint32_t v; std::memcpy(&v, b, 4); return v; }
            case P_F32: { float v; std::memcpy(&v, b, 4); return v; }
            case P_F64: { double v; std::memcpy(&v, b, 8); return v; }
            default: ok = false; return 0;
        }
    }
};
}  // namespace

bool load_ply(const std::string& path, PlyData& out, std::string& err) {
    std::string data;
    if (!read_file(path, data)) { err = "cannot open PLY file " + path; return false; }
    size_t hend = data.find("end_header");
    if (data.compare(0, 3, "ply") != 0 || hend == std::string::npos) { err = "not a PLY file: " + path; return false; }
    size_t body = data.find('\n', hend);
    if (body == std::string::npos) { err = "truncated PLY header"; return false; }
    ++body;
    std::istringstream hs(data.substr(0, hend));
    std::string line, fmt;
    std::vector<PElem> elems;
    while (std::getline(hs, line)) {
        std::istringstream ls(line);
        std::string kw;
        ls >> kw;
        if (kw == "format") ls >> fmt;
        else if (kw == "element") { PElem e; ls >> e.name >> e.count; elems.push_back(e); }
        else if (kw == "property" && !elems.empty()) {
            PProp pr; std::string t; ls >> t;
            if (t == "list") {
                std::string ct, it; ls >> ct >> it >> pr.name;
                pr.list = true; pr.count = ptype(ct); pr.type = ptype(it);
            } else { pr.type = ptype(t); ls >> pr.name; }
            if (pr.type == P_BAD || (pr.list && pr.count == P_BAD)) { err = "unsupported PLY property type"; return false; }
            elems.back().props.push_back(pr);
        }
    }
    bool ascii = fmt == "ascii";
    bool big = fmt == "binary_big_endian";
    if (!ascii && !big && fmt != "binary_little_endian") { err = "unsupported PLY format " + fmt; return false; }

    out.positions.clear();
    out.faces.clear();
    BinReader br{(const unsigned char*)data.data() + body, (const unsigned char*)data.data() + data.size(), big};
    std::istringstream as(ascii ? data.substr(body) : std::string());
    auto rd = [&](PType t) -> double {
        if (!ascii) return br.read(t);
        double v = 0; as >> v; if (!as) br.ok = false; return v;
    };
    for (auto& e : elems) {
        bool isv = e.name == "vertex", isf = e.name == "face";
        int xi = -1, yi = -1, zi = -1, fi = -1;
        for (size_t k = 0; k < e.props.size(); ++k) {
            if (e.props[k].name == "x") xi = (int)k;
            if (e.props[k].name == "y") yi = (int)k;
            if (e.props[k].name == "z") zi = (int)k;
            if (e.props[k].list && (e.props[k].name == "vertex_indices" || e.props[k].name == "vertex_index")) fi = (int)k;
        }
        for (size_t i = 0; i < e.count; ++i) {
            std::array<double, 3> pos{0, 0, 0};
            std::vector<int> idx;
            for (size_t k = 0; k < e.props.size(); ++k) {
                const PProp& pr = e.props[k];
                if (pr.list) {
                    size_t n = (size_t)rd(pr.count);
                    for (size_t j = 0; j < n; ++j) {
                        double v = rd(pr.type);
                        if ((int)k == fi) idx.push_back((int)v);
                    }
                } else {
                    double v = rd(pr.type);
                    if ((int)k == xi) pos[0] = v;
                    if ((int)k == yi) pos[1] = v;
                    if ((int)k == zi) pos[2] = v;
                }
            }
            if (!br.ok) { err = "truncated PLY body: " + path; return false; }
            if (isv) out.positions.push_back(pos);
            if (isf && fi >= 0) out.faces.push_back(std::move(idx));
        }
    }
    return true;
}

// ============================================================================
// Images.  stbi_load(filename, &w, &h, &channels, 0) keeps the file's channel
// count and 8-bit values; LDRImage::GetSample reads three consecutive bytes at
// channels*(i + j*width) (LDRImage.h:16-26).
// ============================================================================
namespace {
uint32_t be32(const unsigned char* p) { return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | p[3]; }

bool load_png(const std::string& data, Image8& img, std::string& err) {
    const unsigned char* d = (const unsigned char*)data.data();
    size_t n = data.size();
    static const unsigned char sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    if (n < 8 || std::memcmp(d, sig, 8) != 0) { err = "not a PNG"; return false; }
    size_t p = 8;
    uint32_t w = 0, h = 0; int depth = 0, ctype = 0, interlace = 0;
    std::string idat;
    std::vector<unsigned char> palette, trns;
    while (p + 8 <= n) {
        uint32_t len = be32(d + p);
        std::string type((const char*)d + p + 4, 4);
        if (p + 12 + len > n) { err = "truncated PNG"; return false; }
        const unsigned char* c = d + p + 8;
        if (type == "IHDR") {
            if (len < 13) { err = "bad PNG header"; return false; }
            w = be32(c); h = be32(c + 4); depth = c[8]; ctype = c[9]; interlace = c[12];
        } else if (type == "PLTE") palette.assign(c, c + len);
        else if (type == "tRNS") trns.assign(c, c + len);
        else if (type == "IDAT") idat.append((const char*)c, len);
        else if (type == "IEND") break;
        p += 12 + len;
    }
    if (!w || !h) { err = "PNG without IHDR"; return false; }
    if (interlace) { err = "interlaced PNG not supported"; return false; }
    int samples = ctype == 0 ? 1 : ctype == 2 ? 3 : ctype == 3 ? 1 : ctype == 4 ? 2 : ctype == 6 ? 4 : 0;
    if (!samples) { err = "bad PNG colour type"; return false; }
    if (w > 65536 || h > 65536) { err = "PNG too large"; return false; }
    const bool depth_ok = depth == 8 || (depth == 16 && ctype != 3) ||
                          ((depth == 1 || depth == 2 || depth == 4) && (ctype == 0 || ctype == 3));
    if (!depth_ok) { err = "bad PNG bit depth"; return false; }
    size_t bpp_bits = size_t(samples) * depth;
    size_t stride = (w * bpp_bits + 7) / 8;
    size_t bpp = std::max<size_t>(1, bpp_bits / 8);
    std::vector<unsigned char> raw((stride + 1) * h);
    uLongf rawlen = raw.size();
    if (uncompress(raw.data(), &rawlen, (const Bytef*)idat.data(), idat.size()) != Z_OK || rawlen != raw.size()) {
        err = "PNG inflate failed"; return false;
    }
    std::vector<unsigned char> px(stride * h), prev(stride, 0);
    for (uint32_t y = 0; y < h; ++y) {
        const unsigned char* src = &raw[y * (stride + 1)];
        unsigned char* cur = &px[y * stride];
        int f = src[0];
        ++src;
        for (size_t x = 0; x < stride; ++x) {
            int a = x >= bpp ? cur[x - bpp] : 0, b = prev[x], cc = x >= bpp ? prev[x - bpp] : 0;
            int v = src[x];
            switch (f) {
                case 0: break;
                case 1: v += a; break;
                case 2: v += b; break;
                case 3: v += (a + b) / 2; break;
                case 4: { int pp = a + b - cc, pa = std::abs(pp - a), pb = std::abs(pp - b), pc = std::abs(pp - cc);
                          v += (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : cc); break; }
                default: err = "bad PNG filter"; return false;
            }
            cur[x] = (unsigned char)v;
        }
        std::memcpy(prev.data(), cur, stride);
    }
    // expand to 8-bit samples; palette -> RGB(A) like stbi
    int outc = ctype == 3 ? (trns.empty() ? 3 : 4) : samples;
    img.width = (int)w; img.height = (int)h; img.channels = outc;
    img.data.assign(size_t(w) * h * outc, 0);
    for (uint32_t y = 0; y < h; ++y) {
        const unsigned char* row = &px[y * stride];
        for (uint32_t x = 0; x < w; ++x) {
            for (int s = 0; s < samples; ++s) {
                size_t sidx = size_t(x) * samples + s;
                int v;
                if (depth == 8) v = row[sidx];
                else if (depth == 16) v = row[sidx * 2];   // stbi keeps the high byte
                else {
                    size_t bit = sidx * depth;
                    int raw_v = (row[bit / 8] >> (8 - depth - bit % 8)) & ((1 << depth) - 1);
                    v = ctype == 3 ? raw_v : raw_v * 255 / ((1 << depth) - 1);
                }
                if (ctype == 3) {
                    size_t pi = size_t(v) * 3;
                    unsigned char* o = &img.data[(size_t(y) * w + x) * outc];
                    if (pi + 2 < palette.size()) { o[0] = palette[pi]; o[1] = palette[pi + 1]; o[2] = palette[pi + 2]; }
                    if (outc == 4) o[3] = size_t(v) < trns.size() ? trns[v] : 255;
                } else {
                    img.data[(size_t(y) * w + x) * outc + s] = (unsigned char)v;
                }
            }
        }
    }
    return true;
}

bool load_pnm(const std::string& data, Image8& img, std::string& err) {
    std::istringstream s(data);
    std::string magic;
    s >> magic;
    auto next_int = [&](int& v) {
        while (true) {
            s >> std::ws;
            if (s.peek() == '#') { std::string c; std::getline(s, c); continue; }
            s >> v; return bool(s);
        }
    };
    int w, h, mx;
    if (!next_int(w) || !next_int(h) || !next_int(mx)) { err = "bad PNM header"; return false; }
    int ch = (magic == "P6" || magic == "P3") ? 3 : (magic == "P5" || magic == "P2") ? 1 : 0;
    if (!ch || mx <= 0 || mx > 255) { err = "unsupported PNM variant " + magic; return false; }
    img.width = w; img.height = h; img.channels = ch;
    img.data.resize(size_t(w) * h * ch);
    if (magic == "P6" || magic == "P5") {
        s.get();   // single whitespace after maxval
        s.read((char*)img.data.data(), img.data.size());
        if ((size_t)s.gcount() != img.data.size()) { err = "truncated PNM"; return false; }
    } else {
        for (auto& b : img.data) { int v; if (!(s >> v)) { err = "truncated PNM"; return false; } b = (unsigned char)v; }
    }
    return true;
}
}  // namespace

bool load_image8(const std::string& path, Image8& img, std::string& err) {
    std::string data;
    if (!read_file(path, data)) { err = "cannot open image " + path; return false; }
    if (data.size() >= 8 && (unsigned char)data[0] == 137 && data[1] == 'P' && data[2] == 'N' && data[3] == 'G')
        return load_png(data, img, err);
    if (data.size() >= 2 && data[0] == 'P' && data[1] >= '1' && data[1] <= '6') return load_pnm(data, img, err);
    err = "unsupported image format (PNG / PPM / PGM only): " + path;
    return false;
}

// ============================================================================
// OpenEXR images (replaces tinyexr's LoadEXR as HDRImage.h:45-72 uses it): single-part
// scanline files, compression NONE / RLE / ZIPS / ZIP, HALF or FLOAT samples.  LoadEXR's
// behaviour kept: the R, G, B, A channels are looked for among the first four channels of the
// (name-sorted) channel list, a single-channel image is replicated into R, G, B, A, alpha
// defaults to 1, HALF samples are widened exactly, and a file with lineOrder != 0 comes out
// flipped vertically (tinyexr places line y at height-1-y for decreasing order).  HDRImage
// keeps R, G, B.  Tiled, multi-part, deep and PIZ / PXR24 / B44 / DWA files are refused.
// ============================================================================
namespace {
float half_to_float(uint16_t h) {
    const uint32_t sign = uint32_t(h >> 15) << 31;
    const int ex = (h >> 10) & 31;
    uint32_t man = h & 1023u;
    uint32_t bits;
    if (ex == 0) {
        if (man == 0) {
            bits = sign;
        } else {                                  // subnormal half: normalise
            int e = -1;
            do { ++e; man <<= 1; } while (!(man & 1024u));
            bits = sign | (uint32_t(127 - 15 - e) << 23) | ((man & 1023u) << 13);
        }
    } else if (ex == 31) {
        bits = sign | 0x7F800000u | (man << 13);
    } else {
        bits = sign | (uint32_t(ex - 15 + 127) << 23) | (man << 13);
    }
    float f;
    std::memcpy(&f, &bits, 4);
    return f;
}

// OpenEXR's byte reordering + delta predictor undone (ZIP and RLE share it; ImfZip.cpp)
void exr_unpredict(std::vector<unsigned char>& t, unsigned char* dst) {
    for (size_t i = 1; i < t.size(); ++i) t[i] = (unsigned char)(int(t[i - 1]) + int(t[i]) - 128);
    const size_t n = t.size(), half = (n + 1) / 2;
    for (size_t i = 0, a = 0, b = half; i < n;) {
        dst[i++] = t[a++];
        if (i < n) dst[i++] = t[b++];
    }
}

bool exr_rle(const unsigned char* in, size_t inLen, std::vector<unsigned char>& out) {
    size_t o = 0;
    while (inLen > 0) {
        const int c = (signed char)*in;
        if (c < 0) {
            const size_t n = size_t(-c);
            if (inLen < n + 1 || o + n > out.size()) return false;
            std::memcpy(&out[o], in + 1, n);
            o += n; in += n + 1; inLen -= n + 1;
        } else {
            const size_t n = size_t(c) + 1;
            if (inLen < 2 || o + n > out.size()) return false;
            std::memset(&out[o], in[1], n);
            o += n; in += 2; inLen -= 2;
        }
    }
    return o == out.size();
}

template <typename T> T rd(const unsigned char* p) { T v; std::memcpy(&v, p, sizeof(T)); return v; }
}  // namespace

bool load_exr(const std::string& path, int& width, int& height, std::vector<float>& rgb, std::string& err) {
    std::string file;
    if (!read_file(path, file)) { err = "cannot open image " + path; return false; }
    const unsigned char* d = (const unsigned char*)file.data();
    const size_t n = file.size();
    if (n < 8 || rd<uint32_t>(d) != 20000630u) { err = "not an OpenEXR file: " + path; return false; }
    const uint32_t ver = rd<uint32_t>(d + 4);
    if ((ver & 0xFF) != 2 || (ver & 0x1A00)) { err = "tiled / multi-part / deep EXR not supported: " + path; return false; }
    struct Chan { std::string name; int type; };
    std::vector<Chan> chans;
    int comp = -1, lineOrder = 0;
    int32_t dw[4] = {0, 0, -1, -1};
    size_t p = 8;
    auto cstr = [&](std::string& s) {
        const size_t e = file.find('\0', p);
        if (e == std::string::npos) return false;
        s.assign(file, p, e - p);
        p = e + 1;
        return true;
    };
    while (true) {
        std::string name, type;
        if (!cstr(name)) { err = "truncated EXR header"; return false; }
        if (name.empty()) break;
        if (!cstr(type) || p + 4 > n) { err = "truncated EXR header"; return false; }
        const uint32_t sz = rd<uint32_t>(d + p);
        p += 4;
        if (p + sz > n) { err = "truncated EXR header"; return false; }
        const unsigned char* v = d + p;
        if (name == "channels") {
            size_t q = 0;
            while (q < sz && v[q]) {
                const char* nm = (const char*)v + q;
                const size_t L = std::strlen(nm);
                q += L + 1;
                if (q + 16 > sz) { err = "bad EXR channel list"; return false; }
                chans.push_back({std::string(nm, L), rd<int32_t>(v + q)});
                if (rd<int32_t>(v + q + 8) != 1 || rd<int32_t>(v + q + 12) != 1) {
                    err = "subsampled EXR channels not supported"; return false;
                }
                q += 16;
            }
        } else if (name == "compression") {
            if (sz < 1) { err = "bad EXR compression attribute"; return false; }
            comp = v[0];
        } else if (name == "dataWindow") {
            if (sz < 16) { err = "bad EXR dataWindow attribute"; return false; }
            for (int k = 0; k < 4; ++k) dw[k] = rd<int32_t>(v + 4 * k);
        } else if (name == "lineOrder") {
            if (sz < 1) { err = "bad EXR lineOrder attribute"; return false; }
            lineOrder = v[0];
        }
        p += sz;
    }
    const int64_t w64 = int64_t(dw[2]) - dw[0] + 1, h64 = int64_t(dw[3]) - dw[1] + 1;
    if (chans.empty() || w64 <= 0 || h64 <= 0) { err = "EXR without channels / data window"; return false; }
    if (w64 > (1 << 16) || h64 > (1 << 16) || w64 * h64 > (int64_t(1) << 28)) { err = "EXR data window too large"; return false; }
    width = int(w64);
    height = int(h64);
    int lines;
    switch (comp) {
        case 0: case 1: case 2: lines = 1; break;      // NONE, RLE, ZIPS
        case 3: lines = 16; break;                     // ZIP
        default: err = "EXR compression " + std::to_string(comp) + " not supported (NONE/RLE/ZIPS/ZIP)"; return false;
    }
    size_t pixBytes = 0;
    std::vector<size_t> choff;
    for (const Chan& c : chans) {
        if (c.type != 1 && c.type != 2) { err = "EXR UINT channels not supported"; return false; }
        choff.push_back(pixBytes);
        pixBytes += c.type == 1 ? 2 : 4;
    }
    // LoadEXR: R/G/B/A among the first four channels; one channel -> grey
    int iR = -1, iG = -1, iB = -1, iA = -1;
    for (size_t c = 0; c < chans.size() && c < 4; ++c) {
        if (chans[c].name == "R") iR = (int)c;
        else if (chans[c].name == "G") iG = (int)c;
        else if (chans[c].name == "B") iB = (int)c;
        else if (chans[c].name == "A") iA = (int)c;
    }
    if (chans.size() == 1) iR = iG = iB = 0;
    else if (iR < 0 || iG < 0 || iB < 0) { err = "EXR without R, G, B channels: " + path; return false; }
    (void)iA;
    const int nblocks = (height + lines - 1) / lines;
    if (p + size_t(nblocks) * 8 > n) { err = "truncated EXR offset table"; return false; }
    rgb.assign(size_t(width) * height * 3, 0.f);
    std::vector<unsigned char> raw, tmp;
    for (int b = 0; b < nblocks; ++b) {
        const uint64_t off = rd<uint64_t>(d + p + 8 * size_t(b));
        // subtractions, not sums: a 64-bit offset near 2^64 must not wrap past the check
        if (off > n || n - off < 8) { err = "bad EXR chunk offset"; return false; }
        const int y = rd<int32_t>(d + off);
        const uint32_t len = rd<uint32_t>(d + off + 4);
        if (len > n - off - 8) { err = "truncated EXR chunk"; return false; }
        const int64_t line0_64 = int64_t(y) - dw[1];
        if (line0_64 < 0 || line0_64 >= height) { err = "bad EXR chunk line"; return false; }
        const int line0 = int(line0_64);
        const int nl = std::min(lines, height - line0);
        if (line0 < 0 || nl <= 0) { err = "bad EXR chunk line"; return false; }
        const size_t need = size_t(nl) * width * pixBytes;
        const unsigned char* src = d + off + 8;
        raw.resize(need);
        if (comp == 0 || len == need) {                 // stored (also a chunk that did not compress)
            if (len != need) { err = "bad EXR chunk size"; return false; }
            std::memcpy(raw.data(), src, need);
        } else if (comp == 1) {
            tmp.assign(need, 0);
            if (!exr_rle(src, len, tmp)) { err = "EXR RLE decode failed"; return false; }
            exr_unpredict(tmp, raw.data());
        } else {
            tmp.assign(need, 0);
            uLongf outLen = need;
            if (uncompress(tmp.data(), &outLen, src, len) != Z_OK || outLen != need) { err = "EXR inflate failed"; return false; }
            exr_unpredict(tmp, raw.data());
        }
        for (int v = 0; v < nl; ++v) {
            const int row = lineOrder == 0 ? line0 + v : height - 1 - (line0 + v);
            const unsigned char* lineBase = raw.data() + size_t(v) * width * pixBytes;
            const int ci[3] = {iR, iG, iB};
            for (int k = 0; k < 3; ++k) {
                const Chan& c = chans[ci[k]];
                const unsigned char* cb = lineBase + choff[ci[k]] * width;
                for (int x = 0; x < width; ++x) {
                    const float f = c.type == 1 ? half_to_float(rd<uint16_t>(cb + 2 * size_t(x))) : rd<float>(cb + 4 * size_t(x));
                    rgb[3 * (size_t(row) * width + x) + k] = f;
                }
            }
        }
    }
    return true;
}

// ============================================================================
// Writers (main.cpp:187-195 uses stbi_write_png / stbi_write_hdr)
// ============================================================================
static void put32(std::string& s, uint32_t v) {
    s += char(v >> 24); s += char(v >> 16); s += char(v >> 8); s += char(v);
}
static void chunk(std::string& out, const char* type, const std::string& body) {
    put32(out, (uint32_t)body.size());
    std::string tb = std::string(type, 4) + body;
    out += tb;
    put32(out, (uint32_t)crc32(0, (const Bytef*)tb.data(), (uInt)tb.size()));
}

bool write_png(const std::string& path, int w, int h, const unsigned char* rgb, std::string& err) {
    std::string raw;
    raw.reserve(size_t(h) * (size_t(w) * 3 + 1));
    for (int y = 0; y < h; ++y) { raw += char(0); raw.append((const char*)rgb + size_t(y) * w * 3, size_t(w) * 3); }
    uLongf zlen = compressBound(raw.size());
    std::string z(zlen, '\0');
    if (compress2((Bytef*)&z[0], &zlen, (const Bytef*)raw.data(), raw.size(), 6) != Z_OK) { err = "zlib failure"; return false; }
    z.resize(zlen);
    std::string out("\x89PNG\r\n\x1a\n", 8), ihdr;
    put32(ihdr, w); put32(ihdr, h);
    ihdr += char(8); ihdr += char(2); ihdr += char(0); ihdr += char(0); ihdr += char(0);
    chunk(out, "IHDR", ihdr);
    chunk(out, "IDAT", z);
    chunk(out, "IEND", std::string());
    std::ofstream f(path, std::ios::binary);
    if (!f) { err = "cannot write " + path; return false; }
    f.write(out.data(), out.size());
    return bool(f);
}

bool write_hdr(const std::string& path, int w, int h, const float* rgb, std::string& err) {
    std::ofstream f(path, std::ios::binary);
    if (!f) { err = "cannot write " + path; return false; }
    f << "#?RADIANCE\nFORMAT=32-bit_rle_rgbe\n\n-Y " << h << " +X " << w << "\n";
    std::string row;
    for (int y = 0; y < h; ++y) {
        row.clear();
        for (int x = 0; x < w; ++x) {
            const float* c = rgb + (size_t(y) * w + x) * 3;
            float m = std::max(c[0], std::max(c[1], c[2]));
            unsigned char e[4] = {0, 0, 0, 0};
            if (m >= 1e-32f) {
                int ex;
                float scale = std::frexp(m, &ex) * 256.0f / m;
                e[0] = (unsigned char)(c[0] * scale); e[1] = (unsigned char)(c[1] * scale);
                e[2] = (unsigned char)(c[2] * scale); e[3] = (unsigned char)(ex + 128);
            }
            row.append((const char*)e, 4);
        }
        f.write(row.data(), row.size());
    }
    return bool(f);
}

}  // namespace rtg
