// scene_loader.cpp — host-side scene input: the YAML scene
// files of the reference -> descriptor tables for rt_scene_upload().
//
// Semantics restated from ray-tracer-cli/src/scene_loader.rs (SceneParser):
//   process_definitions 46-62   `define:` entries by name suffix, in order
//   parse_color         64-90   hash {color|value}, [r,g,b], or a name
//   parse_material      92-149  name | {extend?, value?, fields...}
//   parse_pattern       151-193 stripes/gradient/rings/checkers
//   parse_transformation 195-238 ops LEFT-multiply, a named transform
//                                RIGHT-multiplies (quirk kept)
//   parse_scene         249-335 camera/light/plane/sphere/cube/cone/cylinder;
//                                unknown `add:` kinds are ignored
//   parse_f64           338-344 Integer -> f64, Real -> str::parse, else error
// YAML scalars are resolved the way yaml-rust 0.4.5 does (the reference's
// parser, Cargo.lock), for the subset the scene files use: block sequences
// and mappings, flow sequences/mappings, plain and quoted scalars, comments.
// Anchors, aliases, tags, block scalars and multi-document streams are
// rejected loudly instead of being misread.
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/rtc_scene.h"
#include "host_math.hpp"
#include "rtc_internal.hpp"
#include "shape_identity.hpp"

namespace rtc {
namespace {

using hm::M4;

// ------------------------------------------------------------------ YAML
struct Node {
    enum Kind { Bad, Null, Bool, Int, Real, Str, Seq, Map } kind = Bad;
    bool b = false;
    int64_t i = 0;
    std::string s;  // Real keeps its source text (scene_loader.rs:341 parses it)
    std::vector<Node> seq;
    std::vector<std::pair<std::string, Node>> map;

    const Node& operator[](const std::string& key) const {  // yaml-rust Index<&str>
        static const Node bad;
        if (kind != Map) return bad;
        const Node* hit = &bad;
        for (const auto& kv : map)
            if (kv.first == key) hit = &kv.second;  // a repeated key: the last one wins
        return *hit;
    }
    bool is_bad() const { return kind == Bad; }
};

[[noreturn]] void fail(const std::string& msg) { throw std::runtime_error(msg); }

// Rust `str::parse::<f64>` grammar: [+-]? (inf|infinity|nan | digits[.digits?] | .digits) ([eE][+-]?digits)?
bool rust_parse_f64(const std::string& v, double& out) {
    std::string t = v;
    size_t p = 0;
    if (p < t.size() && (t[p] == '+' || t[p] == '-')) ++p;
    std::string rest = t.substr(p);
    std::string low;
    for (char c : rest) low += (char)std::tolower((unsigned char)c);
    if (low == "inf" || low == "infinity" || low == "nan") {
        double r = (low == "nan") ? NAN : INFINITY;
        out = (t[0] == '-') ? -r : r;
        return true;
    }
    size_t q = p, digits = 0;
    while (q < t.size() && std::isdigit((unsigned char)t[q])) ++q, ++digits;
    if (q < t.size() && t[q] == '.') {
        ++q;
        while (q < t.size() && std::isdigit((unsigned char)t[q])) ++q, ++digits;
    }
    if (digits == 0) return false;
    if (q < t.size() && (t[q] == 'e' || t[q] == 'E')) {
        ++q;
        if (q < t.size() && (t[q] == '+' || t[q] == '-')) ++q;
        size_t e = 0;
        while (q < t.size() && std::isdigit((unsigned char)t[q])) ++q, ++e;
        if (e == 0) return false;
    }
    if (q != t.size()) return false;
    errno = 0;
    out = std::strtod(t.c_str(), nullptr);  // correctly rounded, as Rust's parser
    return true;
}

bool rust_parse_i64(const std::string& v, int64_t& out) {
    if (v.empty()) return false;
    size_t p = (v[0] == '+' || v[0] == '-') ? 1 : 0;
    if (p == v.size()) return false;
    for (size_t k = p; k < v.size(); ++k)
        if (!std::isdigit((unsigned char)v[k])) return false;
    errno = 0;
    long long r = std::strtoll(v.c_str(), nullptr, 10);
    if (errno == ERANGE) return false;
    out = r;
    return true;
}

// yaml-rust 0.4.5 Yaml::from_str for a plain scalar
Node resolve_plain(const std::string& v) {
    Node n;
    int64_t iv;
    if (v.rfind("0x", 0) == 0) {
        char* end = nullptr;
        errno = 0;
        long long r = std::strtoll(v.c_str() + 2, &end, 16);
        if (v.size() > 2 && *end == 0 && errno == 0) {
            n.kind = Node::Int;
            n.i = r;
            return n;
        }
    }
    if (v.rfind("0o", 0) == 0) {
        char* end = nullptr;
        errno = 0;
        long long r = std::strtoll(v.c_str() + 2, &end, 8);
        if (v.size() > 2 && *end == 0 && errno == 0) {
            n.kind = Node::Int;
            n.i = r;
            return n;
        }
    }
    if (v == "~" || v == "null") {
        n.kind = Node::Null;
        return n;
    }
    if (v == "true" || v == "false") {
        n.kind = Node::Bool;
        n.b = (v == "true");
        return n;
    }
    if (rust_parse_i64(v, iv)) {
        n.kind = Node::Int;
        n.i = iv;
        return n;
    }
    double dv;
    if (v == ".inf" || v == ".Inf" || v == ".INF" || v == "+.inf" || v == "+.Inf" || v == "+.INF" || v == "-.inf" ||
        v == "-.Inf" || v == "-.INF" || v == ".nan" || v == "NaN" || v == ".NAN" || rust_parse_f64(v, dv)) {
        n.kind = Node::Real;
        n.s = v;
        return n;
    }
    n.kind = Node::Str;
    n.s = v;
    return n;
}

struct Line {
    int indent;
    std::string text;
    int lineno;
};

// Strip a comment: '#' at line start or after whitespace, outside quotes.
std::string strip_comment(const std::string& s) {
    char q = 0;
    for (size_t k = 0; k < s.size(); ++k) {
        char c = s[k];
        if (q) {
            if (c == q) q = 0;
            continue;
        }
        if (c == '\'' || c == '"') q = c;
        else if (c == '#' && (k == 0 || s[k - 1] == ' ' || s[k - 1] == '\t')) return s.substr(0, k);
    }
    return s;
}
std::string rtrim(const std::string& s) {
    size_t e = s.size();
    while (e > 0 && (s[e - 1] == ' ' || s[e - 1] == '\t' || s[e - 1] == '\r')) --e;
    return s.substr(0, e);
}
std::string trim(const std::string& s) {
    size_t b = 0;
    while (b < s.size() && (s[b] == ' ' || s[b] == '\t')) ++b;
    return rtrim(s.substr(b));
}

class Parser {
public:
    explicit Parser(const std::string& text) {
        std::istringstream in(text);
        std::string raw;
        int no = 0;
        bool doc_started = false;
        while (std::getline(in, raw)) {
            ++no;
            if (raw.find('\t') != std::string::npos && raw.find_first_not_of(" \t") != std::string::npos &&
                raw.find_first_not_of(' ') < raw.size() && raw[raw.find_first_not_of(' ')] == '\t')
                fail("line " + std::to_string(no) + ": tab indentation is not valid YAML");
            std::string s = rtrim(strip_comment(raw));
            if (trim(s).empty()) continue;
            if (s == "---") {
                if (doc_started || !lines_.empty()) fail("multiple YAML documents (scene_loader.rs:357 expects one)");
                doc_started = true;
                continue;
            }
            if (s == "...") break;
            int ind = 0;
            while (ind < (int)s.size() && s[ind] == ' ') ++ind;
            lines_.push_back({ind, s.substr(ind), no});
        }
    }
    Node parse_document() {
        size_t i = 0;
        // yaml-rust yields no document for an empty stream and the reference
        // asserts exactly one (scene_loader.rs:357)
        if (lines_.empty()) fail("empty YAML stream (scene_loader.rs:357 expects one document)");
        Node n = block(i, lines_[0].indent);
        if (i != lines_.size()) fail("line " + std::to_string(lines_[i].lineno) + ": unexpected content");
        return n;
    }

private:
    std::vector<Line> lines_;

    static bool is_seq_item(const std::string& t) { return t == "-" || t.rfind("- ", 0) == 0; }

    // Position of the ':' separating a mapping key, or npos.
    static size_t key_colon(const std::string& t) {
        if (t.empty() || t[0] == '[' || t[0] == '{') return std::string::npos;
        char q = 0;
        int depth = 0;
        for (size_t k = 0; k < t.size(); ++k) {
            char c = t[k];
            if (q) {
                if (c == q) q = 0;
                continue;
            }
            if (c == '\'' || c == '"') q = c;
            else if (c == '[' || c == '{') ++depth;
            else if (c == ']' || c == '}') --depth;
            else if (c == ':' && depth == 0 && (k + 1 == t.size() || t[k + 1] == ' ')) return k;
        }
        return std::string::npos;
    }

    static void reject_unsupported(const std::string& v, int lineno) {
        if (v.empty()) return;
        char c = v[0];
        if (c == '&' || c == '*' || c == '!' || c == '|' || c == '>' || c == '%' || c == '@' || c == '`')
            fail("line " + std::to_string(lineno) + ": unsupported YAML construct '" + v + "'");
    }

    Node scalar_text(const std::string& raw, int lineno) {
        std::string v = trim(raw);
        reject_unsupported(v, lineno);
        Node n;
        if (!v.empty() && (v[0] == '"' || v[0] == '\'')) {
            char q = v[0];
            if (v.size() < 2 || v.back() != q) fail("line " + std::to_string(lineno) + ": unterminated quoted scalar");
            std::string body = v.substr(1, v.size() - 2), out;
            for (size_t k = 0; k < body.size(); ++k) {
                if (q == '"' && body[k] == '\\' && k + 1 < body.size()) {
                    char e = body[++k];
                    out += (e == 'n') ? '\n' : (e == 't') ? '\t' : e;
                } else if (q == '\'' && body[k] == '\'' && k + 1 < body.size() && body[k + 1] == '\'') {
                    out += '\'';
                    ++k;
                } else {
                    out += body[k];
                }
            }
            n.kind = Node::Str;
            n.s = out;
            return n;
        }
        if (v.empty()) {
            n.kind = Node::Null;
            return n;
        }
        return resolve_plain(v);
    }

    // ---- flow collections: [a, b, [c]] and {k: v}
    Node flow(const std::string& t, size_t& p, int lineno) {
        auto skip = [&]() {
            while (p < t.size() && (t[p] == ' ')) ++p;
        };
        skip();
        if (p >= t.size()) fail("line " + std::to_string(lineno) + ": truncated flow collection");
        if (t[p] == '[' || t[p] == '{') {
            const char close = (t[p] == '[') ? ']' : '}';
            const bool is_map = (t[p] == '{');
            ++p;
            Node n;
            n.kind = is_map ? Node::Map : Node::Seq;
            skip();
            if (p < t.size() && t[p] == close) {
                ++p;
                return n;
            }
            for (;;) {
                if (is_map) {
                    size_t k0 = p;
                    while (p < t.size() && t[p] != ':' && t[p] != ',' && t[p] != '}') ++p;
                    if (p >= t.size() || t[p] != ':') fail("line " + std::to_string(lineno) + ": bad flow mapping");
                    std::string key = trim(t.substr(k0, p - k0));
                    if (key.size() >= 2 && (key[0] == '"' || key[0] == '\'')) key = key.substr(1, key.size() - 2);
                    ++p;
                    n.map.emplace_back(key, flow(t, p, lineno));
                } else {
                    n.seq.push_back(flow(t, p, lineno));
                }
                skip();
                if (p < t.size() && t[p] == ',') {
                    ++p;
                    skip();
                    if (p < t.size() && t[p] == close) {  // trailing comma
                        ++p;
                        return n;
                    }
                    continue;
                }
                if (p < t.size() && t[p] == close) {
                    ++p;
                    return n;
                }
                fail("line " + std::to_string(lineno) + ": malformed flow collection");
            }
        }
        size_t b = p;
        char q = 0;
        if (t[p] == '"' || t[p] == '\'') {
            q = t[p++];
            while (p < t.size() && t[p] != q) ++p;
            if (p < t.size()) ++p;
        } else {
            while (p < t.size() && t[p] != ',' && t[p] != ']' && t[p] != '}') ++p;
        }
        return scalar_text(t.substr(b, p - b), lineno);
    }

    Node flow_value(size_t& i, const std::string& first, int lineno) {
        // A flow collection may continue on following lines until balanced.
        std::string t = first;
        auto balanced = [](const std::string& s) {
            int d = 0;
            char q = 0;
            for (char c : s) {
                if (q) {
                    if (c == q) q = 0;
                    continue;
                }
                if (c == '\'' || c == '"') q = c;
                else if (c == '[' || c == '{') ++d;
                else if (c == ']' || c == '}') --d;
            }
            return d <= 0;
        };
        while (!balanced(t)) {
            if (i >= lines_.size()) fail("line " + std::to_string(lineno) + ": unterminated flow collection");
            t += " " + lines_[i++].text;
        }
        size_t p = 0;
        Node n = flow(t, p, lineno);
        while (p < t.size() && t[p] == ' ') ++p;
        if (p != t.size()) fail("line " + std::to_string(lineno) + ": trailing characters after flow collection");
        return n;
    }

    Node value_text(size_t& i, const std::string& v, int lineno) {
        std::string t = trim(v);
        if (!t.empty() && (t[0] == '[' || t[0] == '{')) return flow_value(i, t, lineno);
        return scalar_text(t, lineno);
    }

    Node block(size_t& i, int indent) {
        const Line& L = lines_[i];
        if (L.indent != indent) fail("line " + std::to_string(L.lineno) + ": bad indentation");
        if (is_seq_item(L.text)) return sequence(i, indent);
        if (key_colon(L.text) != std::string::npos) return mapping(i, indent);
        ++i;
        return value_text(i, L.text, L.lineno);
    }

    // value of "key:" or "-" with nothing after it on the line
    Node nested(size_t& i, int parent_indent, bool allow_same_indent_seq) {
        if (i < lines_.size()) {
            const Line& N = lines_[i];
            if (N.indent > parent_indent) return block(i, N.indent);
            if (allow_same_indent_seq && N.indent == parent_indent && is_seq_item(N.text))
                return sequence(i, parent_indent);
        }
        Node n;
        n.kind = Node::Null;
        return n;
    }

    Node sequence(size_t& i, int indent) {
        Node n;
        n.kind = Node::Seq;
        while (i < lines_.size() && lines_[i].indent == indent && is_seq_item(lines_[i].text)) {
            Line L = lines_[i];
            size_t off = 1;
            while (off < L.text.size() && L.text[off] == ' ') ++off;
            std::string rest = L.text.substr(off);
            if (rest.empty()) {
                ++i;
                n.seq.push_back(nested(i, indent, false));
            } else if (is_seq_item(rest) || key_colon(rest) != std::string::npos) {
                // "- key: v" / "- - x": an inline block collection at column indent+off
                lines_[i].indent = indent + (int)off;
                lines_[i].text = rest;
                n.seq.push_back(block(i, indent + (int)off));
            } else {
                ++i;
                n.seq.push_back(value_text(i, rest, L.lineno));
            }
        }
        return n;
    }

    Node mapping(size_t& i, int indent) {
        Node n;
        n.kind = Node::Map;
        while (i < lines_.size() && lines_[i].indent == indent && !is_seq_item(lines_[i].text)) {
            const Line L = lines_[i];
            size_t c = key_colon(L.text);
            if (c == std::string::npos) fail("line " + std::to_string(L.lineno) + ": expected 'key: value'");
            std::string key = trim(L.text.substr(0, c));
            reject_unsupported(key, L.lineno);
            if (key.size() >= 2 && (key[0] == '"' || key[0] == '\'')) key = key.substr(1, key.size() - 2);
            std::string v = trim(L.text.substr(c + 1));
            ++i;
            if (v.empty())
                n.map.emplace_back(key, nested(i, indent, true));
            else
                n.map.emplace_back(key, value_text(i, v, L.lineno));
        }
        return n;
    }
};

// ----------------------------------------------------------- SceneParser
struct Color3 {
    double v[3];
};

struct MaterialV {  // composites/material.rs:8-20 with the pattern as a table index
    double color[3] = {1, 1, 1};
    int pattern = -1;
    double ambient = 0.1, diffuse = 0.9, specular = 0.9, shininess = 200.0;
    double reflectiveness = 0.0, transparency = 0.0, refractive_index = 1.0;
    bool casts_shadow = true;
};

double parse_f64(const Node& n, const char* what) {  // scene_loader.rs:338-344
    if (n.kind == Node::Int) return (double)n.i;
    if (n.kind == Node::Real) {
        double v;
        if (!rust_parse_f64(n.s, v)) fail(std::string("invalid float literal for ") + what + ": '" + n.s + "'");
        return v;
    }
    fail(std::string("expected a number for ") + what);
}

void parse_array_of_3(const std::vector<Node>& v, size_t from, double out[3], const char* what) {  // 346-352
    if (v.size() < from + 3) fail(std::string("expected 3 numbers for ") + what);
    for (int k = 0; k < 3; ++k) out[k] = parse_f64(v[from + k], what);
}

const std::vector<Node>& as_vec(const Node& n, const char* what) {
    if (n.kind != Node::Seq) fail(std::string("expected a sequence for ") + what);
    return n.seq;
}

class SceneParser {
public:
    std::vector<rt_pattern_desc> patterns;

    void process_definitions(const Node& doc) {  // 46-62
        if (doc.kind != Node::Seq) return;
        for (const Node& entry : doc.seq) {
            const Node& d = entry["define"];
            if (d.kind != Node::Str) continue;
            const std::string& name = d.s;
            auto ends = [&](const char* suf) {
                size_t l = std::strlen(suf);
                return name.size() >= l && name.compare(name.size() - l, l, suf) == 0;
            };
            if (ends("-color"))
                colors_[name] = parse_color(entry);
            else if (ends("-material"))
                materials_[name] = parse_material(entry);
            else if (ends("-transform") || ends("-object"))
                transforms_[name] = parse_transformation(entry);
        }
    }

    Color3 parse_color(const Node& y) const {  // 64-90
        switch (y.kind) {
            case Node::Map:
                return parse_color(!y["color"].is_bad() ? y["color"] : y["value"]);
            case Node::Seq: {
                Color3 c;
                parse_array_of_3(y.seq, 0, c.v, "color");
                return c;
            }
            case Node::Str: {
                auto it = colors_.find(y.s);
                if (it == colors_.end()) fail("unknown color '" + y.s + "'");
                return it->second;
            }
            default:
                fail("Incorrect color value");
        }
    }

    MaterialV parse_material(const Node& y0) {  // 92-149
        if (y0.kind == Node::Str) {
            auto it = materials_.find(y0.s);
            if (it == materials_.end()) fail("unknown material '" + y0.s + "'");
            return it->second;
        }
        MaterialV m;
        if (!y0["extend"].is_bad()) {
            const Node& e = y0["extend"];
            if (e.kind != Node::Str) fail("material extend must name a material");
            auto it = materials_.find(e.s);
            if (it == materials_.end()) fail("unknown material '" + e.s + "'");
            m = it->second;
        }
        const Node& y = !y0["value"].is_bad() ? y0["value"] : y0;
        if (!y["color"].is_bad()) {
            Color3 c = parse_color(y["color"]);
            for (int k = 0; k < 3; ++k) m.color[k] = c.v[k];
        }
        if (!y["pattern"].is_bad()) m.pattern = parse_pattern(y["pattern"]);
        if (!y["ambient"].is_bad()) m.ambient = parse_f64(y["ambient"], "ambient");
        if (!y["diffuse"].is_bad()) m.diffuse = parse_f64(y["diffuse"], "diffuse");
        if (!y["specular"].is_bad()) m.specular = parse_f64(y["specular"], "specular");
        if (!y["shininess"].is_bad()) m.shininess = parse_f64(y["shininess"], "shininess");
        if (!y["reflective"].is_bad()) m.reflectiveness = parse_f64(y["reflective"], "reflective");
        if (!y["transparency"].is_bad()) m.transparency = parse_f64(y["transparency"], "transparency");
        if (!y["refractive-index"].is_bad()) m.refractive_index = parse_f64(y["refractive-index"], "refractive-index");
        if (y["casts-shadow"].kind == Node::Bool) m.casts_shadow = y["casts-shadow"].b;
        return m;
    }

    int parse_pattern(const Node& y) {  // 151-193
        const std::vector<Node>& colors = as_vec(y["colors"], "pattern colors");
        if (colors.size() < 2) fail("a pattern needs two colors");
        Color3 a = parse_color(colors[0]);
        Color3 b = parse_color(colors[1]);
        M4 t = hm::identity();
        bool has_t = !y["transform"].is_bad();
        if (has_t) t = parse_transformation(y["transform"]);
        const Node& ty = y["type"];
        if (ty.kind != Node::Str) fail("Incorrect pattern type");
        rt_pattern_desc d{};
        if (ty.s == "stripes") d.kind = RT_PATTERN_STRIPE;
        else if (ty.s == "gradient") d.kind = RT_PATTERN_GRADIENT;
        else if (ty.s == "rings") d.kind = RT_PATTERN_RING;
        else if (ty.s == "checkers") d.kind = RT_PATTERN_CHECKER;
        else fail("Incorrect pattern type '" + ty.s + "'");
        d.sub_a = d.sub_b = -1;
        for (int k = 0; k < 3; ++k) {
            d.color_a[k] = a.v[k];
            d.color_b[k] = b.v[k];
        }
        // Pattern::new starts at IDENTITY; set_transformation stores inverse()
        M4 inv = has_t ? hm::inverse(t) : hm::identity();
        for (int r = 0; r < 4; ++r)
            for (int c = 0; c < 4; ++c) d.inverse[4 * r + c] = inv.m[r][c];
        patterns.push_back(d);
        return (int)patterns.size() - 1;
    }

    M4 parse_transformation(const Node& y0) const {  // 195-238
        M4 t = hm::identity();
        const Node& y = !y0["value"].is_bad() ? y0["value"] : y0;
        if (y.kind != Node::Seq) return t;  // Yaml::into_iter of a non-array is empty
        for (const Node& op : y.seq) {
            if (op.kind == Node::Str) {
                auto it = transforms_.find(op.s);
                if (it == transforms_.end()) fail("unknown transform '" + op.s + "'");
                t = hm::mul(t, it->second);  // named: right-multiplied
            } else if (op.kind == Node::Seq) {
                if (op.seq.empty() || op.seq[0].kind != Node::Str) fail("transform op must start with its name");
                const std::string& name = op.seq[0].s;
                double v[3];
                if (name == "scale") {
                    parse_array_of_3(op.seq, 1, v, "scale");
                    t = hm::mul(hm::scaling(v[0], v[1], v[2]), t);
                } else if (name == "translate") {
                    parse_array_of_3(op.seq, 1, v, "translate");
                    t = hm::mul(hm::translation(v[0], v[1], v[2]), t);
                } else if (name == "rotate-x" || name == "rotate-y" || name == "rotate-z") {
                    if (op.seq.size() < 2) fail("rotation needs an angle");
                    double a = parse_f64(op.seq[1], name.c_str());
                    t = hm::mul(hm::rotation(name[7] - 'x', a), t);
                }  // unknown op: ignored (scene_loader.rs:232)
            }
        }
        return t;
    }

    void parse_scene(const Node& doc, std::vector<rt_shape_desc>& shapes, std::vector<MaterialV>& shape_materials,
                     std::vector<rt_light_desc>& lights, rt_camera_desc& camera) {  // 249-335
        camera_zero(camera);
        if (doc.kind != Node::Seq) return;
        for (const Node& entry : doc.seq) {
            const Node& add = entry["add"];
            if (add.kind != Node::Str) continue;
            const std::string& what = add.s;
            if (what == "camera") {
                double w = parse_f64(entry["width"], "width");
                double h = parse_f64(entry["height"], "height");
                double fov = parse_f64(entry["field-of-view"], "field-of-view");
                double from[3], to[3], up[3];
                parse_array_of_3(as_vec(entry["from"], "from"), 0, from, "from");
                parse_array_of_3(as_vec(entry["to"], "to"), 0, to, "to");
                parse_array_of_3(as_vec(entry["up"], "up"), 0, up, "up");
                rt_camera_make(sat_u32(w), sat_u32(h), fov, from, to, up, &camera);
            } else if (what == "light") {
                rt_light_desc l{};
                parse_array_of_3(as_vec(entry["at"], "light at"), 0, l.position, "light at");
                parse_array_of_3(as_vec(entry["intensity"], "light intensity"), 0, l.intensity, "intensity");
                lights.push_back(l);
            } else if (what == "plane" || what == "sphere" || what == "cube" || what == "cone" || what == "cylinder") {
                MaterialV m = parse_material(entry["material"]);
                M4 t = parse_transformation(entry["transform"]);
                rt_shape_desc s{};
                s.kind = what == "sphere"  ? RT_SHAPE_SPHERE
                         : what == "plane" ? RT_SHAPE_PLANE
                         : what == "cube"  ? RT_SHAPE_CUBE
                         : what == "cone"  ? RT_SHAPE_CONE
                                           : RT_SHAPE_CYLINDER;
                M4 inv = hm::inverse(t);
                for (int r = 0; r < 4; ++r)
                    for (int c = 0; c < 4; ++c) s.inverse[4 * r + c] = inv.m[r][c];
                s.minimum = -DBL_MAX;  // Cylinder/Cone::default, cylinder.rs:133-141
                s.maximum = DBL_MAX;
                s.closed = 0;
                if (s.kind == RT_SHAPE_CONE || s.kind == RT_SHAPE_CYLINDER) {
                    if (entry["closed"].kind == Node::Bool) s.closed = entry["closed"].b ? 1 : 0;
                    if (!entry["max"].is_bad()) s.maximum = parse_f64(entry["max"], "max");
                    if (!entry["min"].is_bad()) s.minimum = parse_f64(entry["min"], "min");
                }
                shapes.push_back(s);
                shape_materials.push_back(m);
            }  // other kinds ignored (scene_loader.rs:330)
        }
    }

    static uint32_t sat_u32(double v) {  // f64 `as u32`
        if (!(v > 0)) return 0;
        if (v >= 4294967295.0) return 4294967295u;
        return (uint32_t)v;
    }
    static void camera_zero(rt_camera_desc& c) {  // Camera::new(0, 0, 0), scene_loader.rs:251
        std::memset(&c, 0, sizeof(c));
        for (int k = 0; k < 4; ++k) c.inverse[5 * k] = 1.0;
        hm::CameraSize s = hm::camera_size(0, 0, 0.0);
        c.half_width = s.half_width;
        c.half_height = s.half_height;
        c.pixel_size = s.pixel_size;
    }

private:
    std::map<std::string, Color3> colors_;
    std::map<std::string, MaterialV> materials_;
    std::map<std::string, M4> transforms_;
};

bool material_value_eq(const rt_material_desc& a, const rt_material_desc& b) {
    return std::memcmp(&a, &b, sizeof(a)) == 0;
}

}  // namespace

struct SceneTables {
    std::vector<rt_shape_desc> shapes;
    std::vector<rt_material_desc> materials;
    std::vector<rt_pattern_desc> patterns;
    std::vector<rt_light_desc> lights;
    rt_camera_desc camera{};
    uint32_t duplicates = 0;
};

static void load_text(const std::string& text, SceneTables& out) {
    Parser p(text);
    Node doc = p.parse_document();
    SceneParser sp;
    sp.process_definitions(doc);
    std::vector<MaterialV> shape_mats;
    sp.parse_scene(doc, out.shapes, shape_mats, out.lights, out.camera);
    out.patterns = sp.patterns;
    // material table: one entry per distinct material value
    for (size_t k = 0; k < out.shapes.size(); ++k) {
        const MaterialV& m = shape_mats[k];
        rt_material_desc d{};
        for (int c = 0; c < 3; ++c) d.color[c] = m.color[c];
        d.ambient = m.ambient;
        d.diffuse = m.diffuse;
        d.specular = m.specular;
        d.shininess = m.shininess;
        d.reflectiveness = m.reflectiveness;
        d.transparency = m.transparency;
        d.refractive_index = m.refractive_index;
        d.casts_shadow = m.casts_shadow ? 1 : 0;
        d.pattern = m.pattern;
        int idx = -1;
        for (size_t j = 0; j < out.materials.size(); ++j)
            if (material_value_eq(out.materials[j], d)) idx = (int)j;
        if (idx < 0) {
            out.materials.push_back(d);
            idx = (int)out.materials.size() - 1;
        }
        out.shapes[k].material = idx;
    }
    // shapes equal by value to an earlier one (shape.rs:34-38); rt_scene_upload
    // gives such shapes one identity class, as the containers walk does
    std::vector<uint32_t> cls;
    out.duplicates = ident::shape_classes(out.shapes.data(), (uint32_t)out.shapes.size(), out.materials.data(),
                                          out.patterns.data(), cls);
}

}  // namespace rtc

struct rt_scene {
    rtc::SceneTables t;
};

extern "C" {

int rt_scene_load_yaml_text(const char* text, rt_scene** out) {
    if (!text || !out) return rtc::set_error(RT_ERR_INVALID, "rt_scene_load_yaml_text: null argument");
    try {
        auto s = std::make_unique<rt_scene>();
        rtc::load_text(text, s->t);
        *out = s.release();
        return RT_OK;
    } catch (const std::exception& e) {
        return rtc::set_error(RT_ERR_IO, std::string("scene: ") + e.what());
    }
}

int rt_scene_load_yaml(const char* path, rt_scene** out) {
    if (!path || !out) return rtc::set_error(RT_ERR_INVALID, "rt_scene_load_yaml: null argument");
    std::ifstream f(path, std::ios::binary);
    if (!f) return rtc::set_error(RT_ERR_IO, std::string("cannot open scene file ") + path);
    std::stringstream ss;
    ss << f.rdbuf();
    return rt_scene_load_yaml_text(ss.str().c_str(), out);
}

int rt_scene_view_get(const rt_scene* s, rt_scene_view* v) {
    if (!s || !v) return rtc::set_error(RT_ERR_INVALID, "rt_scene_view_get: null argument");
    v->shapes = s->t.shapes.data();
    v->n_shapes = (uint32_t)s->t.shapes.size();
    v->materials = s->t.materials.data();
    v->n_materials = (uint32_t)s->t.materials.size();
    v->patterns = s->t.patterns.data();
    v->n_patterns = (uint32_t)s->t.patterns.size();
    v->lights = s->t.lights.data();
    v->n_lights = (uint32_t)s->t.lights.size();
    v->camera = s->t.camera;
    v->duplicate_shapes = s->t.duplicates;
    return RT_OK;
}

void rt_scene_free(rt_scene* s) { delete s; }

int rt_camera_make(uint32_t width, uint32_t height, double fov, const double from[3], const double to[3],
                   const double up[3], rt_camera_desc* out) {
    if (!from || !to || !up || !out) return rtc::set_error(RT_ERR_INVALID, "rt_camera_make: null argument");
    using namespace rtc::hm;
    rtc::hm::CameraSize s = camera_size(width, height, fov);
    M4 inv = inverse(view_transform(from, to, up));
    out->width = width;
    out->height = height;
    out->field_of_view = fov;
    out->half_width = s.half_width;
    out->half_height = s.half_height;
    out->pixel_size = s.pixel_size;
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c) out->inverse[4 * r + c] = inv.m[r][c];
    const double o[3] = {0, 0, 0};
    mul_point(inv, o, out->origin);  // camera.rs:114-116
    return RT_OK;
}

int rt_camera_resize(rt_camera_desc* cam, uint32_t width, uint32_t height) {
    if (!cam) return rtc::set_error(RT_ERR_INVALID, "rt_camera_resize: null argument");
    rtc::hm::CameraSize s = rtc::hm::camera_size(width, height, cam->field_of_view);
    cam->width = width;
    cam->height = height;
    cam->half_width = s.half_width;
    cam->half_height = s.half_height;
    cam->pixel_size = s.pixel_size;
    return RT_OK;
}

int rt_camera_set_transform(rt_camera_desc* cam, const double t[16]) {
    if (!cam || !t) return rtc::set_error(RT_ERR_INVALID, "rt_camera_set_transform: null argument");
    rtc::hm::M4 a;
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c) a.m[r][c] = t[4 * r + c];
    const rtc::hm::M4 inv = rtc::hm::inverse(a);  // camera.rs:124-127
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c) cam->inverse[4 * r + c] = inv.m[r][c];
    const double o[3] = {0, 0, 0};
    rtc::hm::mul_point(inv, o, cam->origin);  // update_origin, camera.rs:114-116
    return RT_OK;
}

int rt_matrix_inverse(const double m[16], double out[16]) {
    if (!m || !out) return rtc::set_error(RT_ERR_INVALID, "rt_matrix_inverse: null argument");
    rtc::hm::M4 a;
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c) a.m[r][c] = m[4 * r + c];
    rtc::hm::M4 inv = rtc::hm::inverse(a);
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c) out[4 * r + c] = inv.m[r][c];
    return RT_OK;
}

}  // extern "C"
