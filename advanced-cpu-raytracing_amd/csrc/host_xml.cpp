// XML DOM (tinyxml2-compatible text-node rules) and std::stringstream emulation.
// See host_xml.hpp for the reference behaviour each piece reproduces.
#include "host_xml.hpp"

#include <cerrno>
#include <climits>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <limits>
#include <sstream>

namespace rtg {

// ============================================================================
// DOM
// ============================================================================
const char* XmlNode::GetText() const {
    if (!children.empty() && children[0]->kind == Text) return children[0]->value.c_str();
    return nullptr;
}

XmlNode* XmlNode::FirstChildElement(const char* nm) const {
    for (auto& c : children)
        if (c->kind == Element && (!nm || c->name == nm)) return c.get();
    return nullptr;
}

XmlNode* XmlNode::NextSiblingElement(const char* nm) const {
    if (!parent) return nullptr;
    bool seen = false;
    for (auto& c : parent->children) {
        if (seen && c->kind == Element && (!nm || c->name == nm)) return c.get();
        if (c.get() == this) seen = true;
    }
    return nullptr;
}

const char* XmlNode::Attribute(const char* nm, const char* val) const {
    for (auto& a : attrs) {
        if (a.first == nm) {
            if (!val) return a.second.c_str();
            return a.second == val ? a.second.c_str() : nullptr;
        }
    }
    return nullptr;
}

namespace {

inline bool is_ws(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }
inline bool is_name_char(char c) {
    unsigned char u = (unsigned char)c;
    return std::isalnum(u) || c == '_' || c == ':' || c == '.' || c == '-' || u >= 0x80;
}

void append_utf8(std::string& out, unsigned long cp) {
    if (cp < 0x80) out += char(cp);
    else if (cp < 0x800) { out += char(0xC0 | (cp >> 6)); out += char(0x80 | (cp & 0x3F)); }
    else if (cp < 0x10000) {
        out += char(0xE0 | (cp >> 12)); out += char(0x80 | ((cp >> 6) & 0x3F));
        out += char(0x80 | (cp & 0x3F));
    } else {
        out += char(0xF0 | (cp >> 18)); out += char(0x80 | ((cp >> 12) & 0x3F));
        out += char(0x80 | ((cp >> 6) & 0x3F)); out += char(0x80 | (cp & 0x3F));
    }
}

// newline normalisation + entity decoding (StrPair::GetStr, tinyxml2.cpp:~260-360)
std::string decode(const std::string& raw, bool entities) {
    std::string out;
    out.reserve(raw.size());
    for (size_t i = 0; i < raw.size(); ++i) {
        char c = raw[i];
        if (c == '\r') {
            out += '\n';
            if (i + 1 < raw.size() && raw[i + 1] == '\n') ++i;
            continue;
        }
        if (entities && c == '&') {
            size_t semi = raw.find(';', i);
            if (semi != std::string::npos && semi - i <= 10) {
                std::string ent = raw.substr(i + 1, semi - i - 1);
                bool ok = true;
                if (ent == "amp") out += '&';
                else if (ent == "lt") out += '<';
                else if (ent == "gt") out += '>';
                else if (ent == "quot") out += '"';
                else if (ent == "apos") out += '\'';
                else if (ent.size() > 1 && ent[0] == '#') {
                    unsigned long cp = (ent[1] == 'x' || ent[1] == 'X')
                                           ? std::strtoul(ent.c_str() + 2, nullptr, 16)
                                           : std::strtoul(ent.c_str() + 1, nullptr, 10);
                    append_utf8(out, cp);
                } else ok = false;
                if (ok) { i = semi; continue; }
            }
        }
        out += c;
    }
    return out;
}

struct Parser {
    const std::string& s;
    size_t p = 0;
    std::string err;
    explicit Parser(const std::string& str) : s(str) {}

    bool starts(const char* lit) const { return s.compare(p, std::strlen(lit), lit) == 0; }

    // parse children of `parent` until `</closing>` (or EOF for the document)
    bool parse_children(XmlNode* parent, const std::string& closing) {
        for (;;) {
            size_t start = p;
            while (p < s.size() && is_ws(s[p])) ++p;
            if (p >= s.size()) {
                if (!closing.empty()) { err = "unexpected end of file inside <" + closing + ">"; return false; }
                return true;
            }
            if (starts("</")) {
                p += 2;
                size_t ns = p;
                while (p < s.size() && is_name_char(s[p])) ++p;
                std::string nm = s.substr(ns, p - ns);
                while (p < s.size() && is_ws(s[p])) ++p;
                if (p >= s.size() || s[p] != '>') { err = "malformed closing tag"; return false; }
                ++p;
                if (nm != closing) { err = "mismatched closing tag </" + nm + ">"; return false; }
                return true;
            }
            auto node = std::make_unique<XmlNode>();
            node->parent = parent;
            if (starts("<?")) {
                size_t e = s.find("?>", p);
                if (e == std::string::npos) { err = "unterminated declaration"; return false; }
                node->kind = XmlNode::Other; p = e + 2;
            } else if (starts("<!--")) {
                size_t e = s.find("-->", p + 4);
                if (e == std::string::npos) { err = "unterminated comment"; return false; }
                node->kind = XmlNode::Comment; p = e + 3;
            } else if (starts("<![CDATA[")) {
                size_t e = s.find("]]>", p + 9);
                if (e == std::string::npos) { err = "unterminated CDATA"; return false; }
                node->kind = XmlNode::Text;
                node->value = decode(s.substr(p + 9, e - p - 9), false);
                p = e + 3;
            } else if (starts("<!")) {
                size_t e = s.find('>', p);
                if (e == std::string::npos) { err = "unterminated <!"; return false; }
                node->kind = XmlNode::Other; p = e + 1;
            } else if (s[p] == '<') {
                ++p;
                node->kind = XmlNode::Element;
                size_t ns = p;
                while (p < s.size() && is_name_char(s[p])) ++p;
                node->name = s.substr(ns, p - ns);
                if (node->name.empty()) { err = "empty element name"; return false; }
                bool closed = false;
                for (;;) {
                    while (p < s.size() && is_ws(s[p])) ++p;
                    if (p >= s.size()) { err = "unterminated start tag"; return false; }
                    if (s[p] == '/') {
                        if (p + 1 >= s.size() || s[p + 1] != '>') { err = "bad '/'"; return false; }
                        p += 2; closed = true; break;
                    }
                    if (s[p] == '>') { ++p; break; }
                    size_t as = p;
                    while (p < s.size() && is_name_char(s[p])) ++p;
                    std::string an = s.substr(as, p - as);
                    if (an.empty()) { err = "bad attribute"; return false; }
                    while (p < s.size() && is_ws(s[p])) ++p;
                    if (p >= s.size() || s[p] != '=') { err = "attribute without value"; return false; }
                    ++p;
                    while (p < s.size() && is_ws(s[p])) ++p;
                    if (p >= s.size() || (s[p] != '"' && s[p] != '\'')) { err = "unquoted attribute"; return false; }
                    char q = s[p++];
                    size_t ve = s.find(q, p);
                    if (ve == std::string::npos) { err = "unterminated attribute"; return false; }
                    node->attrs.emplace_back(an, decode(s.substr(p, ve - p), true));
                    p = ve + 1;
                }
                if (!closed) {
                    if (!parse_children(node.get(), node->name)) return false;
                }
            } else {
                // text: everything from `start` (leading whitespace included) to '<'
                node->kind = XmlNode::Text;
                size_t e = s.find('<', p);
                if (e == std::string::npos) e = s.size();
                node->value = decode(s.substr(start, e - start), true);
                p = e;
            }
            parent->children.push_back(std::move(node));
        }
    }
};

}  // namespace

bool XmlDocument::Parse(const std::string& text) {
    doc = std::make_unique<XmlNode>();
    doc->kind = XmlNode::Other;
    Parser ps(text);
    if (!ps.parse_children(doc.get(), "")) {
        error = ps.err;
        return false;
    }
    return true;
}

bool XmlDocument::Load(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) { error = "cannot open " + path; return false; }
    std::stringstream ss;
    ss << f.rdbuf();
    return Parse(ss.str());
}

XmlNode* XmlDocument::FirstChild() const {
    // The reference takes the first node as <Scene>; a leading <?xml?> or comment
    // makes every later lookup dereference null there.  Skipping non-elements is the
    // one deliberate leniency of this loader.
    if (!doc) return nullptr;
    for (auto& c : doc->children)
        if (c->kind == XmlNode::Element) return c.get();
    return nullptr;
}

// ============================================================================
// RefStream
// ============================================================================
RefStream& RefStream::put(const char* s) {
    if (!s) { bad_ = true; return *this; }
    if (!good()) { fail_ = true; return *this; }
    buf_ += s;
    return *this;
}

RefStream& RefStream::endl() {
    if (!good()) { fail_ = true; return *this; }
    buf_ += '\n';
    return *this;
}

bool RefStream::sentry_in() {
    if (!good()) { fail_ = true; return false; }
    while (pos_ < buf_.size() && std::isspace((unsigned char)buf_[pos_])) ++pos_;
    if (pos_ >= buf_.size()) { eof_ = true; fail_ = true; return false; }
    return true;
}

// num_get accumulation (libstdc++ locale_facets.tcc _M_extract_int/_M_extract_float)
std::string RefStream::numeric_run(bool allow_float) {
    std::string acc;
    auto at_end = [&]() { if (pos_ >= buf_.size()) { eof_ = true; return true; } return false; };
    if (at_end()) return acc;
    char c = buf_[pos_];
    if (c == '+' || c == '-') { acc += c; ++pos_; }
    bool seen_digit = false, seen_point = false;
    while (!at_end()) {
        c = buf_[pos_];
        if (c >= '0' && c <= '9') { acc += c; seen_digit = true; ++pos_; }
        else if (allow_float && c == '.' && !seen_point) { acc += c; seen_point = true; ++pos_; }
        else break;
    }
    if (allow_float && seen_digit && !at_end() && (buf_[pos_] == 'e' || buf_[pos_] == 'E')) {
        acc += buf_[pos_++];
        if (!at_end() && (buf_[pos_] == '+' || buf_[pos_] == '-')) acc += buf_[pos_++];
        while (!at_end() && buf_[pos_] >= '0' && buf_[pos_] <= '9') acc += buf_[pos_++];
    }
    return acc;
}

RefStream& RefStream::get(int& v) {
    if (!sentry_in()) return *this;
    std::string acc = numeric_run(false);
    bool has_digit = false;
    for (char c : acc) has_digit |= (c >= '0' && c <= '9');
    if (!has_digit) { v = 0; fail_ = true; return *this; }
    errno = 0;
    long long x = std::strtoll(acc.c_str(), nullptr, 10);
    if (errno == ERANGE || x > INT_MAX) { v = INT_MAX; fail_ = true; }
    else if (x < INT_MIN) { v = INT_MIN; fail_ = true; }
    else v = (int)x;
    return *this;
}

template <typename T>
static void convert_float(const std::string& acc, T& v, bool& fail) {
    char* end = nullptr;
    errno = 0;
    T x;
    if (sizeof(T) == sizeof(float)) x = (T)std::strtof(acc.c_str(), &end);
    else x = (T)std::strtod(acc.c_str(), &end);
    if (acc.empty() || end == acc.c_str() || *end != '\0') { v = 0; fail = true; return; }
    if (std::isinf(x)) {
        v = x > 0 ? std::numeric_limits<T>::max() : -std::numeric_limits<T>::max();
        fail = true;
        return;
    }
    v = x;
}

RefStream& RefStream::get(float& v) {
    if (!sentry_in()) return *this;
    convert_float<float>(numeric_run(true), v, fail_);
    return *this;
}

RefStream& RefStream::get(double& v) {
    if (!sentry_in()) return *this;
    convert_float<double>(numeric_run(true), v, fail_);
    return *this;
}

RefStream& RefStream::get(std::string& v) {
    if (!sentry_in()) return *this;
    v.clear();
    while (pos_ < buf_.size() && !std::isspace((unsigned char)buf_[pos_])) v += buf_[pos_++];
    if (pos_ >= buf_.size()) eof_ = true;
    if (v.empty()) fail_ = true;
    return *this;
}

}  // namespace rtg
