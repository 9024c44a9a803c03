// Minimal XML DOM + std::stringstream-extraction emulator used by the scene loader.
//
// The reference parses scenes with tinyxml2 4.0.1 (src/tinyxml2.*) and pulls every
// value out through ONE long-lived std::stringstream per parse function
// (e.g. parser.cpp:29, 878, 989, 1116, 1284, 1503).  Values are appended with
// `stream << text << std::endl` and extracted with `>>`, so leftover tokens, eof and
// fail bits carry from one element to the next.  Results depend on those details
// (e.g. `while (!(stream >> x).eof())` loops at parser.cpp:270 and :1449), so this
// file reproduces them rather than using a tokenizer.
#pragma once

#include <memory>
#include <string>
#include <vector>

namespace rtg {

// ---- DOM ------------------------------------------------------------------
// Node model follows tinyxml2: whitespace-only runs between markup produce no
// node (XMLDocument::Identify skips whitespace and only backs up for real text,
// tinyxml2.cpp:651-716); a text node keeps its leading/trailing whitespace, with
// CR/CRLF normalised to LF and entities decoded (StrPair::GetStr).
struct XmlNode {
    enum Kind { Element, Text, Comment, Other } kind = Other;
    std::string name;                                      // element name
    std::string value;                                     // text value
    std::vector<std::pair<std::string, std::string>> attrs;
    std::vector<std::unique_ptr<XmlNode>> children;
    XmlNode* parent = nullptr;

    // XMLElement::GetText (tinyxml2.cpp:1532): first child if it is text, else null.
    const char* GetText() const;
    // XMLNode::FirstChildElement / NextSiblingElement (name==nullptr: any element).
    XmlNode* FirstChildElement(const char* name = nullptr) const;
    XmlNode* NextSiblingElement(const char* name = nullptr) const;
    // XMLElement::Attribute(name, value): value==nullptr -> attribute value or null;
    // otherwise non-null only when the attribute equals `value`.
    const char* Attribute(const char* name, const char* value = nullptr) const;
};

struct XmlDocument {
    std::unique_ptr<XmlNode> doc;   // synthetic document node
    std::string error;
    bool Load(const std::string& path);
    bool Parse(const std::string& text);
    // The reference uses file.FirstChild() as the scene root (parser.cpp:38).
    XmlNode* FirstChild() const;
};

// ---- std::stringstream emulation -------------------------------------------
// Implements the libstdc++ semantics the parser relies on:
//  * operator<< through a sentry: appends only while good(); a null `const char*`
//    sets badbit (so `stream << elem->GetText()` on an empty element poisons the
//    stream until clear()).
//  * operator>> through a sentry: fails unless good(); skips whitespace, sets
//    eof|fail when the buffer is exhausted; numbers follow num_get (longest
//    sign/digits/point/exponent run, then strtol/strtof/strtod with failbit on
//    garbage or range errors, value 0 / max per C++11); reaching the end of the
//    buffer while reading sets eofbit.
class RefStream {
public:
    RefStream& put(const char* s);          // stream << s
    RefStream& put(const std::string& s) { return put(s.c_str()); }
    RefStream& endl();                      // stream << std::endl
    RefStream& get(int& v);
    RefStream& get(float& v);
    RefStream& get(double& v);
    RefStream& get(std::string& v);
    bool eof() const { return eof_; }
    bool fail() const { return fail_ || bad_; }
    bool good() const { return !eof_ && !fail_ && !bad_; }
    explicit operator bool() const { return !fail(); }
    void clear() { eof_ = fail_ = bad_ = false; }

    // convenience: stream << text << std::endl
    RefStream& line(const char* s) { put(s); if (s) endl(); return *this; }

private:
    bool sentry_in();                       // istream sentry + whitespace skip
    std::string numeric_run(bool allow_float);
    std::string buf_;
    size_t pos_ = 0;
    bool eof_ = false, fail_ = false, bad_ = false;
};

}  // namespace rtg
