// Asset readers for the scene loader: PLY meshes (replaces happly, parser.cpp:1396-1444),
// LDR images (PNG / PNM / JPEG; replaces stb_image as used by LDRImage.h:37-44) and OpenEXR images (replaces
// tinyexr as used by HDRImage.h:45-72).
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
// ----------------------------------------------------------------------------
// JPEG, as stbi_load (stb_image v2.27, vendored by the reference) decodes it: baseline,
// extended and progressive Huffman files, 1 or 3 components, any integer sampling factors.
// The decoded bytes must equal stb's, so its integer algorithms are restated: the
// jidctint-derived IDCT with its fixed-point constants and rounding, the fancy upsamplers
// (v_2, h_2, hv_2 -- the SSE2 kernels stb uses on x86 are bit-identical to these -- and
// nearest for other ratios) with stb's row state machine, and its reduced-precision
// YCbCr->RGB; bit reading follows stb's (a marker ends the data, zeros are fed after it).
// The Huffman decoder is a plain canonical one (stb's 9-bit fast tables give the same
// symbols).  CMYK / YCCK (4 components) and arithmetic coding are refused.
const unsigned char kDezig[64 + 15] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                       12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                       35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                       58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63,
                                       63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};
const uint32_t kBmask[17] = {0, 1, 3, 7, 15, 31, 63, 127, 255, 511, 1023, 2047, 4095, 8191, 16383, 32767, 65535};
const int kJbias[16] = {0, -1, -3, -7, -15, -31, -63, -127, -255, -511, -1023, -2047, -4095, -8191, -16383, -32767};

struct JHuff {
    unsigned char size[257], values[256];
    uint16_t code[256];
    uint32_t maxcode[18];
    int delta[17];
    bool build(const int* count, std::string& err) {
        int k = 0;
        for (int i = 0; i < 16; ++i)
            for (int j = 0; j < count[i]; ++j) {
                if (k >= 256) { err = "bad Huffman table"; return false; }
                size[k++] = (unsigned char)(i + 1);
            }
        size[k] = 0;
        unsigned code_ = 0;
        k = 0;
        int j;
        for (j = 1; j <= 16; ++j) {
            delta[j] = k - (int)code_;
            if (size[k] == j) {
                while (size[k] == j) code[k++] = (uint16_t)(code_++);
                if (code_ - 1 >= (1u << j)) { err = "bad code lengths"; return false; }
            }
            maxcode[j] = code_ << (16 - j);
            code_ <<= 1;
        }
        maxcode[j] = 0xffffffffu;
        return true;
    }
};

struct JComp {
    int id = 0, h = 1, v = 1, tq = 0, hd = 0, ha = 0, dc = 0;
    int x = 0, y = 0, w2 = 0, h2 = 0, coeff_w = 0;
    std::vector<unsigned char> data;
    std::vector<short> coeff;
};

inline unsigned char clamp8(int x) {
    if ((unsigned)x > 255) return x < 0 ? 0 : 255;
    return (unsigned char)x;
}

#define JF2F(x) ((int)(((x) * 4096 + 0.5)))
#define JFSH(x) ((x) * 4096)
// stbi__idct_block (the "islow" integer IDCT), columns then rows
void jidct(unsigned char* out, int stride, const short* data) {
    int val[64];
    auto idct1d = [](int s0, int s1, int s2, int s3, int s4, int s5, int s6, int s7, int& x0, int& x1, int& x2,
                     int& x3, int& t0, int& t1, int& t2, int& t3) {
        int p1, p2, p3, p4, p5;
        p2 = s2; p3 = s6;
        p1 = (p2 + p3) * JF2F(0.5411961f);
        t2 = p1 + p3 * JF2F(-1.847759065f);
        t3 = p1 + p2 * JF2F(0.765366865f);
        p2 = s0; p3 = s4;
        t0 = JFSH(p2 + p3);
        t1 = JFSH(p2 - p3);
        x0 = t0 + t3; x3 = t0 - t3; x1 = t1 + t2; x2 = t1 - t2;
        t0 = s7; t1 = s5; t2 = s3; t3 = s1;
        p3 = t0 + t2; p4 = t1 + t3; p1 = t0 + t3; p2 = t1 + t2;
        p5 = (p3 + p4) * JF2F(1.175875602f);
        t0 = t0 * JF2F(0.298631336f);
        t1 = t1 * JF2F(2.053119869f);
        t2 = t2 * JF2F(3.072711026f);
        t3 = t3 * JF2F(1.501321110f);
        p1 = p5 + p1 * JF2F(-0.899976223f);
        p2 = p5 + p2 * JF2F(-2.562915447f);
        p3 = p3 * JF2F(-1.961570560f);
        p4 = p4 * JF2F(-0.390180644f);
        t3 += p1 + p4; t2 += p2 + p3; t1 += p2 + p4; t0 += p1 + p3;
    };
    for (int i = 0; i < 8; ++i) {
        const short* d = data + i;
        int* v = val + i;
        if (d[8] == 0 && d[16] == 0 && d[24] == 0 && d[32] == 0 && d[40] == 0 && d[48] == 0 && d[56] == 0) {
            const int dc = d[0] * 4;
            v[0] = v[8] = v[16] = v[24] = v[32] = v[40] = v[48] = v[56] = dc;
        } else {
            int x0, x1, x2, x3, t0, t1, t2, t3;
            idct1d(d[0], d[8], d[16], d[24], d[32], d[40], d[48], d[56], x0, x1, x2, x3, t0, t1, t2, t3);
            x0 += 512; x1 += 512; x2 += 512; x3 += 512;
            v[0] = (x0 + t3) >> 10; v[56] = (x0 - t3) >> 10;
            v[8] = (x1 + t2) >> 10; v[48] = (x1 - t2) >> 10;
            v[16] = (x2 + t1) >> 10; v[40] = (x2 - t1) >> 10;
            v[24] = (x3 + t0) >> 10; v[32] = (x3 - t0) >> 10;
        }
    }
    for (int i = 0; i < 8; ++i) {
        const int* v = val + 8 * i;
        unsigned char* o = out + (size_t)i * stride;
        int x0, x1, x2, x3, t0, t1, t2, t3;
        idct1d(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], x0, x1, x2, x3, t0, t1, t2, t3);
        x0 += 65536 + (128 << 17); x1 += 65536 + (128 << 17);
        x2 += 65536 + (128 << 17); x3 += 65536 + (128 << 17);
        o[0] = clamp8((x0 + t3) >> 17); o[7] = clamp8((x0 - t3) >> 17);
        o[1] = clamp8((x1 + t2) >> 17); o[6] = clamp8((x1 - t2) >> 17);
        o[2] = clamp8((x2 + t1) >> 17); o[5] = clamp8((x2 - t1) >> 17);
        o[3] = clamp8((x3 + t0) >> 17); o[4] = clamp8((x3 - t0) >> 17);
    }
}
#undef JF2F
#undef JFSH

struct JpegDec {
    const unsigned char* p;
    const unsigned char* end;
    std::string& err;
    JHuff hdc[4], hac[4];
    uint16_t dequant[4][64] = {};
    JComp comp[4];
    int n = 0, w = 0, h = 0, hmax = 1, vmax = 1, mcux = 0, mcuy = 0, rgb = 0, jfif = 0, app14 = -1;
    bool progressive = false;
    int restart = 0, todo = 0, eob = 0, scan_n = 0, order[4] = {0, 0, 0, 0};
    int ss = 0, se = 0, ah = 0, al = 0;
    uint32_t buf = 0;
    int bits = 0, marker = -1;
    bool nomore = false;
    explicit JpegDec(std::string& e) : err(e) {}
    int get8() { return p < end ? *p++ : 0; }
    int get16() { int a = get8(); return (a << 8) | get8(); }
    bool fail(const char* m) { err = std::string("JPEG: ") + m; return false; }
    void grow() {                                        // stbi__grow_buffer_unsafe
        do {
            unsigned b = nomore ? 0 : (unsigned)get8();
            if (b == 0xff) {
                int c = get8();
                while (c == 0xff) c = get8();
                if (c != 0) { marker = c; nomore = true; return; }
            }
            buf |= b << (24 - bits);
            bits += 8;
        } while (bits <= 24);
    }
    int huff(const JHuff& t) {                           // stbi__jpeg_huff_decode
        if (bits < 16) grow();
        const uint32_t temp = buf >> 16;
        int k = 1;
        while (k <= 16 && !(temp < t.maxcode[k])) ++k;
        if (k == 17) { bits -= 16; return -1; }
        if (k > bits) return -1;
        const int c = (int)((buf >> (32 - k)) & kBmask[k]) + t.delta[k];
        bits -= k;
        buf <<= k;
        return t.values[c];
    }
    int receive(int nb) {                                // stbi__extend_receive
        if (bits < nb) grow();
        const int sgn = (int)(buf >> 31);
        uint32_t k = (buf << nb) | (buf >> ((32 - nb) & 31));
        buf = k & ~kBmask[nb];
        k &= kBmask[nb];
        bits -= nb;
        return (int)k + (kJbias[nb] & (sgn - 1));
    }
    int getbits(int nb) {
        if (bits < nb) grow();
        uint32_t k = (buf << nb) | (buf >> ((32 - nb) & 31));
        buf = k & ~kBmask[nb];
        k &= kBmask[nb];
        bits -= nb;
        return (int)k;
    }
    int getbit() {
        if (bits < 1) grow();
        const uint32_t k = buf;
        buf <<= 1;
        --bits;
        return (int)(k & 0x80000000u) != 0;
    }
    void reset() {
        bits = 0; buf = 0; nomore = false;
        for (auto& c : comp) c.dc = 0;
        marker = -1;
        todo = restart ? restart : 0x7fffffff;
        eob = 0;
    }
    int next_marker() {                                   // stbi__get_marker
        if (marker != -1) { const int m = marker; marker = -1; return m; }
        int x = get8();
        if (x != 0xff) return -1;
        while (x == 0xff) x = get8();
        return x;
    }
    bool block(short* data, JComp& c) {                  // stbi__jpeg_decode_block
        if (bits < 16) grow();
        const int t = huff(hdc[c.hd]);
        if (t < 0 || t > 15) return fail("bad huffman code");
        std::memset(data, 0, 64 * sizeof(short));
        const int diff = t ? receive(t) : 0;
        const int dc = c.dc + diff;
        c.dc = dc;
        const uint16_t* dq = dequant[c.tq];
        data[0] = (short)(dc * dq[0]);
        int k = 1;
        do {
            const int rs = huff(hac[c.ha]);
            if (rs < 0) return fail("bad huffman code");
            const int s = rs & 15, r = rs >> 4;
            if (s == 0) {
                if (rs != 0xf0) break;
                k += 16;
            } else {
                k += r;
                const unsigned zig = kDezig[k++];
                data[zig] = (short)(receive(s) * dq[zig]);
            }
        } while (k < 64);
        return true;
    }
    bool prog_dc(short* data, JComp& c) {
        if (se != 0) return fail("can't merge dc and ac");
        if (bits < 16) grow();
        if (ah == 0) {
            std::memset(data, 0, 64 * sizeof(short));
            const int t = huff(hdc[c.hd]);
            if (t < 0 || t > 15) return fail("can't merge dc and ac");
            const int diff = t ? receive(t) : 0;
            const int dc = c.dc + diff;
            c.dc = dc;
            data[0] = (short)(dc * (1 << al));
        } else if (getbit()) {
            data[0] += (short)(1 << al);
        }
        return true;
    }
    bool prog_ac(short* data, JComp& c) {
        if (ss == 0) return fail("can't merge dc and ac");
        if (ah == 0) {
            if (eob) { --eob; return true; }
            int k = ss;
            do {
                const int rs = huff(hac[c.ha]);
                if (rs < 0) return fail("bad huffman code");
                const int s = rs & 15, r = rs >> 4;
                if (s == 0) {
                    if (r < 15) {
                        eob = 1 << r;
                        if (r) eob += getbits(r);
                        --eob;
                        break;
                    }
                    k += 16;
                } else {
                    k += r;
                    const unsigned zig = kDezig[k++];
                    data[zig] = (short)(receive(s) * (1 << al));
                }
            } while (k <= se);
        } else {
            const short bit = (short)(1 << al);
            if (eob) {
                --eob;
                for (int k = ss; k <= se; ++k) {
                    short* q = &data[kDezig[k]];
                    if (*q != 0 && getbit() && (*q & bit) == 0) *q = (short)(*q > 0 ? *q + bit : *q - bit);
                }
            } else {
                int k = ss;
                do {
                    const int rs = huff(hac[c.ha]);
                    if (rs < 0) return fail("bad huffman code");
                    int s = rs & 15, r = rs >> 4;
                    if (s == 0) {
                        if (r < 15) {
                            eob = (1 << r) - 1;
                            if (r) eob += getbits(r);
                            r = 64;
                        }
                    } else {
                        if (s != 1) return fail("bad huffman code");
                        s = getbit() ? bit : -bit;
                    }
                    while (k <= se) {
                        short* q = &data[kDezig[k++]];
                        if (*q != 0) {
                            if (getbit() && (*q & bit) == 0) *q = (short)(*q > 0 ? *q + bit : *q - bit);
                        } else {
                            if (r == 0) { *q = (short)s; break; }
                            --r;
                        }
                    }
                } while (k <= se);
            }
        }
        return true;
    }
    bool restart_check() {                               // the restart-interval countdown
        if (--todo <= 0) {
            if (bits < 24) grow();
            if (!(marker >= 0xd0 && marker <= 0xd7)) return false;   // not a restart: stop the scan
            reset();
        }
        return true;
    }
    bool entropy() {                                     // stbi__parse_entropy_coded_data
        reset();
        short data[64];
        if (scan_n == 1) {
            JComp& c = comp[order[0]];
            const int bw = (c.x + 7) >> 3, bh = (c.y + 7) >> 3;
            for (int j = 0; j < bh; ++j)
                for (int i = 0; i < bw; ++i) {
                    if (!progressive) {
                        if (!block(data, c)) return false;
                        jidct(&c.data[(size_t)c.w2 * j * 8 + i * 8], c.w2, data);
                    } else {
                        short* cd = &c.coeff[64 * ((size_t)i + (size_t)j * c.coeff_w)];
                        if (!(ss == 0 ? prog_dc(cd, c) : prog_ac(cd, c))) return false;
                    }
                    if (!restart_check()) return true;
                }
            return true;
        }
        for (int j = 0; j < mcuy; ++j)
            for (int i = 0; i < mcux; ++i) {
                for (int k = 0; k < scan_n; ++k) {
                    JComp& c = comp[order[k]];
                    for (int y = 0; y < c.v; ++y)
                        for (int x = 0; x < c.h; ++x) {
                            if (!progressive) {
                                if (!block(data, c)) return false;
                                jidct(&c.data[(size_t)c.w2 * ((j * c.v + y) * 8) + (i * c.h + x) * 8], c.w2, data);
                            } else {
                                short* cd = &c.coeff[64 * ((size_t)(i * c.h + x) + (size_t)(j * c.v + y) * c.coeff_w)];
                                if (!prog_dc(cd, c)) return false;
                            }
                        }
                }
                if (!restart_check()) return true;
            }
        return true;
    }
    bool marker_segment(int m) {                         // stbi__process_marker
        if (m == 0xdd) { if (get16() != 4) return fail("bad DRI len"); restart = get16(); return true; }
        if (m == 0xdb) {
            int L = get16() - 2;
            while (L > 0) {
                const int q = get8(), pr = q >> 4, t = q & 15;
                if ((pr != 0 && pr != 1) || t > 3) return fail("bad DQT");
                for (int i = 0; i < 64; ++i) dequant[t][kDezig[i]] = (uint16_t)(pr ? get16() : get8());
                L -= pr ? 129 : 65;
            }
            return L == 0;
        }
        if (m == 0xc4) {
            int L = get16() - 2;
            while (L > 0) {
                const int q = get8(), tc = q >> 4, th = q & 15;
                if (tc > 1 || th > 3) return fail("bad DHT header");
                int sizes[16], cnt = 0;
                for (int i = 0; i < 16; ++i) { sizes[i] = get8(); cnt += sizes[i]; }
                L -= 17;
                JHuff& t = tc == 0 ? hdc[th] : hac[th];
                if (!t.build(sizes, err)) return false;
                for (int i = 0; i < cnt && i < 256; ++i) t.values[i] = (unsigned char)get8();
                L -= cnt;
            }
            return L == 0;
        }
        if ((m >= 0xe0 && m <= 0xef) || m == 0xfe) {
            int L = get16();
            if (L < 2) return fail("bad APP/COM len");
            L -= 2;
            if (m == 0xe0 && L >= 5) {
                static const unsigned char tag[5] = {'J', 'F', 'I', 'F', 0};
                bool ok = true;
                for (int i = 0; i < 5; ++i) ok &= get8() == tag[i];
                L -= 5;
                if (ok) jfif = 1;
            } else if (m == 0xee && L >= 12) {
                static const unsigned char tag[6] = {'A', 'd', 'o', 'b', 'e', 0};
                bool ok = true;
                for (int i = 0; i < 6; ++i) ok &= get8() == tag[i];
                L -= 6;
                if (ok) { get8(); get16(); get16(); app14 = get8(); L -= 6; }
            }
            p = std::min(end, p + std::max(0, L));
            return true;
        }
        return fail("unknown marker");
    }
    bool frame(int m) {                                  // stbi__process_frame_header
        progressive = m == 0xc2;
        const int Lf = get16();
        if (Lf < 11 || get8() != 8) return fail("8-bit baseline / extended / progressive only");
        h = get16(); w = get16();
        if (!h || !w) return fail("bad size");
        n = get8();
        if (n != 1 && n != 3) return fail("only 1- or 3-component JPEGs are supported");
        if (Lf != 8 + 3 * n) return fail("bad SOF len");
        static const unsigned char rgbId[3] = {'R', 'G', 'B'};
        for (int i = 0; i < n; ++i) {
            comp[i].id = get8();
            if (n == 3 && comp[i].id == rgbId[i]) ++rgb;
            const int q = get8();
            comp[i].h = q >> 4; comp[i].v = q & 15; comp[i].tq = get8();
            if (!comp[i].h || comp[i].h > 4 || !comp[i].v || comp[i].v > 4 || comp[i].tq > 3) return fail("bad component");
        }
        for (int i = 0; i < n; ++i) { hmax = std::max(hmax, comp[i].h); vmax = std::max(vmax, comp[i].v); }
        for (int i = 0; i < n; ++i)
            if (hmax % comp[i].h || vmax % comp[i].v) return fail("fractional sampling");
        mcux = (w + hmax * 8 - 1) / (hmax * 8);
        mcuy = (h + vmax * 8 - 1) / (vmax * 8);
        for (int i = 0; i < n; ++i) {
            JComp& c = comp[i];
            c.x = (w * c.h + hmax - 1) / hmax;
            c.y = (h * c.v + vmax - 1) / vmax;
            c.w2 = mcux * c.h * 8;
            c.h2 = mcuy * c.v * 8;
            c.data.assign((size_t)c.w2 * c.h2, 0);
            if (progressive) { c.coeff_w = c.w2 / 8; c.coeff.assign((size_t)c.w2 * c.h2, 0); }
        }
        return true;
    }
    bool scan_header() {                                 // stbi__process_scan_header
        const int Ls = get16();
        scan_n = get8();
        if (scan_n < 1 || scan_n > 4 || scan_n > n || Ls != 6 + 2 * scan_n) return fail("bad SOS");
        for (int i = 0; i < scan_n; ++i) {
            const int id = get8(), q = get8();
            int which = 0;
            while (which < n && comp[which].id != id) ++which;
            if (which == n) return fail("bad SOS component");
            comp[which].hd = q >> 4; comp[which].ha = q & 15;
            if (comp[which].hd > 3 || comp[which].ha > 3) return fail("bad huff table");
            order[i] = which;
        }
        ss = get8(); se = get8();
        const int aa = get8();
        ah = aa >> 4; al = aa & 15;
        if (progressive) {
            if (ss > 63 || se > 63 || ss > se || ah > 13 || al > 13) return fail("bad SOS");
        } else {
            if (ss != 0 || ah != 0 || al != 0) return fail("bad SOS");
            se = 63;
        }
        return true;
    }
    bool decode() {                                      // stbi__decode_jpeg_image
        if (next_marker() != 0xd8) return fail("no SOI");
        int m = next_marker();
        while (!(m == 0xc0 || m == 0xc1 || m == 0xc2)) {
            if (m == 0xc3 || (m >= 0xc5 && m <= 0xcf && m != 0xc8 && m != 0xcc)) return fail("unsupported coding (lossless / arithmetic)");
            if (!marker_segment(m)) return false;
            m = next_marker();
            while (m == -1) {
                if (p >= end) return fail("no SOF");
                m = next_marker();
            }
        }
        if (!frame(m)) return false;
        m = next_marker();
        while (m != 0xd9) {
            if (m == 0xda) {
                if (!scan_header() || !entropy()) return false;
                if (marker == -1) {
                    while (p < end) {
                        if (get8() == 255) { marker = get8(); break; }
                    }
                }
            } else if (m == 0xdc) {
                if (get16() != 4 || get16() != h) return fail("bad DNL");
            } else if (m == -1) {
                if (p >= end) return fail("no EOI");
            } else if (!marker_segment(m)) {
                return false;
            }
            m = next_marker();
        }
        if (progressive)                                 // stbi__jpeg_finish
            for (int i = 0; i < n; ++i) {
                JComp& c = comp[i];
                const int bw = (c.x + 7) >> 3, bh = (c.y + 7) >> 3;
                for (int j = 0; j < bh; ++j)
                    for (int x = 0; x < bw; ++x) {
                        short* d = &c.coeff[64 * ((size_t)x + (size_t)j * c.coeff_w)];
                        for (int k = 0; k < 64; ++k) d[k] = (short)(d[k] * dequant[c.tq][k]);
                        jidct(&c.data[(size_t)c.w2 * j * 8 + x * 8], c.w2, d);
                    }
            }
        return true;
    }
};

// load_jpeg_image's resample + colour conversion, req_comp = 0 (channels as in the file)
bool load_jpeg(const std::string& data, Image8& img, std::string& err) {
    JpegDec z(err);
    z.p = (const unsigned char*)data.data();
    z.end = z.p + data.size();
    if (!z.decode()) return false;
    const int n = z.n >= 3 ? 3 : 1;
    const bool is_rgb = z.n == 3 && (z.rgb == 3 || (z.app14 == 0 && !z.jfif));
    struct Res { int hs, vs, ystep, wl, ypos; const unsigned char* l0; const unsigned char* l1; std::vector<unsigned char> lb; };
    std::vector<Res> rs(z.n);
    for (int k = 0; k < z.n; ++k) {
        Res& r = rs[k];
        r.hs = z.hmax / z.comp[k].h;
        r.vs = z.vmax / z.comp[k].v;
        r.ystep = r.vs >> 1;
        r.wl = (z.w + r.hs - 1) / r.hs;
        r.ypos = 0;
        r.l0 = r.l1 = z.comp[k].data.data();
        r.lb.assign((size_t)z.w + 3, 0);
    }
    auto resample = [](Res& r, const unsigned char* nr, const unsigned char* fr) -> const unsigned char* {
        unsigned char* out = r.lb.data();
        const int w = r.wl;
        if (r.hs == 1 && r.vs == 1) return nr;
        if (r.hs == 1 && r.vs == 2) {
            for (int i = 0; i < w; ++i) out[i] = (unsigned char)((3 * nr[i] + fr[i] + 2) >> 2);
            return out;
        }
        if (r.hs == 2 && r.vs == 1) {
            if (w == 1) { out[0] = out[1] = nr[0]; return out; }
            out[0] = nr[0];
            out[1] = (unsigned char)((nr[0] * 3 + nr[1] + 2) >> 2);
            int i;
            for (i = 1; i < w - 1; ++i) {
                const int v = 3 * nr[i] + 2;
                out[i * 2] = (unsigned char)((v + nr[i - 1]) >> 2);
                out[i * 2 + 1] = (unsigned char)((v + nr[i + 1]) >> 2);
            }
            out[i * 2] = (unsigned char)((nr[w - 2] * 3 + nr[w - 1] + 2) >> 2);
            out[i * 2 + 1] = nr[w - 1];
            return out;
        }
        if (r.hs == 2 && r.vs == 2) {
            if (w == 1) { out[0] = out[1] = (unsigned char)((3 * nr[0] + fr[0] + 2) >> 2); return out; }
            int t1 = 3 * nr[0] + fr[0];
            out[0] = (unsigned char)((t1 + 2) >> 2);
            for (int i = 1; i < w; ++i) {
                const int t0 = t1;
                t1 = 3 * nr[i] + fr[i];
                out[i * 2 - 1] = (unsigned char)((3 * t0 + t1 + 8) >> 4);
                out[i * 2] = (unsigned char)((3 * t1 + t0 + 8) >> 4);
            }
            out[w * 2 - 1] = (unsigned char)((t1 + 2) >> 2);
            return out;
        }
        for (int i = 0; i < w; ++i)                      // nearest
            for (int j = 0; j < r.hs; ++j) out[i * r.hs + j] = nr[i];
        return out;
    };
    img.width = z.w;
    img.height = z.h;
    img.channels = n;
    img.data.assign((size_t)z.w * z.h * n, 0);
    const unsigned char* co[3] = {nullptr, nullptr, nullptr};
    auto f2f = [](float x) { return ((int)(x * 4096.0f + 0.5f)) << 8; };
    for (int j = 0; j < z.h; ++j) {
        unsigned char* out = &img.data[(size_t)n * z.w * j];
        for (int k = 0; k < z.n; ++k) {
            Res& r = rs[k];
            const bool ybot = r.ystep >= (r.vs >> 1);
            co[k] = resample(r, ybot ? r.l1 : r.l0, ybot ? r.l0 : r.l1);
            if (++r.ystep >= r.vs) {
                r.ystep = 0;
                r.l0 = r.l1;
                if (++r.ypos < z.comp[k].y) r.l1 += z.comp[k].w2;
            }
        }
        if (n == 3) {
            for (int i = 0; i < z.w; ++i) {
                if (is_rgb) {
                    out[3 * i] = co[0][i]; out[3 * i + 1] = co[1][i]; out[3 * i + 2] = co[2][i];
                    continue;
                }
                const int yf = (co[0][i] << 20) + (1 << 19);             // stbi__YCbCr_to_RGB_row
                const int cr = co[2][i] - 128, cb = co[1][i] - 128;
                int R = yf + cr * f2f(1.40200f);
                int G = yf + (cr * -f2f(0.71414f)) + ((cb * -f2f(0.34414f)) & (int)0xffff0000);
                int B = yf + cb * f2f(1.77200f);
                R >>= 20; G >>= 20; B >>= 20;
                out[3 * i] = clamp8(R); out[3 * i + 1] = clamp8(G); out[3 * i + 2] = clamp8(B);
            }
        } else {
            for (int i = 0; i < z.w; ++i) out[i] = co[0][i];
        }
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
    if (data.size() >= 3 && (unsigned char)data[0] == 0xff && (unsigned char)data[1] == 0xd8) return load_jpeg(data, img, err);
    err = "unsupported image format (PNG/PPM/PGM/JPEG only): " + path;
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
            comp = v[0];
        } else if (name == "dataWindow") {
            for (int k = 0; k < 4; ++k) dw[k] = rd<int32_t>(v + 4 * k);
        } else if (name == "lineOrder") {
            lineOrder = v[0];
        }
        p += sz;
    }
    width = dw[2] - dw[0] + 1;
    height = dw[3] - dw[1] + 1;
    if (chans.empty() || width <= 0 || height <= 0) { err = "EXR without channels / data window"; return false; }
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
        if (off + 8 > n) { err = "bad EXR chunk offset"; return false; }
        const int y = rd<int32_t>(d + off);
        const uint32_t len = rd<uint32_t>(d + off + 4);
        if (off + 8 + len > n) { err = "truncated EXR chunk"; return false; }
        const int line0 = y - dw[1];
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
