// pm_support.cpp — Parametrizable, lexical casts and the block-YAML subset.
//
// Parametrizable restates pointmatcher/Parametrizable.cpp:170-240 (defaults,
// min/max bound checks by lexical comparison, parametersUsed bookkeeping);
// the YAML reader replaces the vendored yaml-cpp 0.2 (contrib/yaml-cpp-pm)
// for the block subset the chain files use (doc/Configuration.md:29-60).
#include <cctype>
#include <cstdlib>

#include "pm_core.h"

namespace pm {

// ----------------------------------------------------------- lexical casts --
namespace {
std::string trim(const std::string& s) {
    size_t a = 0, b = s.size();
    while (a < b && std::isspace((unsigned char)s[a])) ++a;
    while (b > a && std::isspace((unsigned char)s[b - 1])) --b;
    return s.substr(a, b - a);
}

template <typename F>
F parse_float(const std::string& raw) {
    const std::string s = trim(raw);
    // Parametrizable.h:48-64: "inf", "-inf", "nan"
    if (s == "inf") return std::numeric_limits<F>::infinity();
    if (s == "-inf") return -std::numeric_limits<F>::infinity();
    if (s == "nan") return std::numeric_limits<F>::quiet_NaN();
    char* end = nullptr;
    const double v = std::strtod(s.c_str(), &end);
    if (s.empty() || end != s.c_str() + s.size()) throw InvalidParameter("bad lexical cast: \"" + s + "\"");
    if (sizeof(F) == 4) {
        // boost::lexical_cast<float> rounds the decimal string directly to float
        return std::strtof(s.c_str(), nullptr);
    }
    return (F)v;
}

template <typename I>
I parse_int(const std::string& raw) {
    const std::string s = trim(raw);
    char* end = nullptr;
    const long long v = std::strtoll(s.c_str(), &end, 10);
    if (s.empty() || end != s.c_str() + s.size()) throw InvalidParameter("bad lexical cast: \"" + s + "\"");
    return (I)v;
}
}  // namespace

template <>
float lexical_cast<float>(const std::string& s) {
    return parse_float<float>(s);
}
template <>
double lexical_cast<double>(const std::string& s) {
    return parse_float<double>(s);
}
template <>
int lexical_cast<int>(const std::string& s) {
    return parse_int<int>(s);
}
template <>
unsigned lexical_cast<unsigned>(const std::string& s) {
    const std::string t = trim(s);
    if (!t.empty() && t[0] == '-') throw InvalidParameter("bad lexical cast: \"" + t + "\"");
    return parse_int<unsigned>(t);
}
template <>
bool lexical_cast<bool>(const std::string& s) {
    const std::string t = trim(s);
    if (t == "1" || t == "true") return true;
    if (t == "0" || t == "false") return false;
    throw InvalidParameter("bad lexical cast: \"" + t + "\"");
}
template <>
std::string lexical_cast<std::string>(const std::string& s) {
    return s;
}

// ---------------------------------------------------------- Parametrizable --
Parametrizable::Parametrizable(const std::string& cn, const ParametersDoc& doc, const Parameters& params)
    : className(cn), parametersDoc(doc) {
    for (const auto& d : parametersDoc) {
        auto it = params.find(d.name);
        if (it != params.end()) {
            const std::string& val = it->second;
            if (d.comp(val, d.minValue))
                throw InvalidParameter("Value " + val + " of parameter " + d.name + " in class " + className +
                                       " is smaller than minimum admissible value " + d.minValue);
            if (d.comp(d.maxValue, val))
                throw InvalidParameter("Value " + val + " of parameter " + d.name + " in class " + className +
                                       " is larger than maximum admissible value " + d.maxValue);
            parameters[d.name] = val;
        } else {
            parameters[d.name] = d.defaultValue;
        }
    }
}

std::string Parametrizable::getParamValueString(const std::string& name) {
    auto it = parameters.find(name);
    if (it == parameters.end())
        throw InvalidParameter("Parameter " + name + " does not exist in class " + className);
    parametersUsed.insert(it->first);
    return it->second;
}

// -------------------------------------------------------------------- YAML --
namespace {
struct Line {
    int indent;
    std::string text;  // trimmed, comment-free
};

std::string strip_comment(const std::string& s) {
    bool sq = false, dq = false;
    for (size_t i = 0; i < s.size(); ++i) {
        const char c = s[i];
        if (c == '\'' && !dq) sq = !sq;
        if (c == '"' && !sq) dq = !dq;
        if (c == '#' && !sq && !dq && (i == 0 || std::isspace((unsigned char)s[i - 1]))) return s.substr(0, i);
    }
    return s;
}

std::string unquote(const std::string& s) {
    if (s.size() >= 2 && ((s.front() == '"' && s.back() == '"') || (s.front() == '\'' && s.back() == '\'')))
        return s.substr(1, s.size() - 2);
    return s;
}

// split "key: value" (value may be empty); returns false when not a mapping
bool split_kv(const std::string& t, std::string& key, std::string& val) {
    bool sq = false, dq = false;
    for (size_t i = 0; i < t.size(); ++i) {
        const char c = t[i];
        if (c == '\'' && !dq) sq = !sq;
        if (c == '"' && !sq) dq = !dq;
        if (c == ':' && !sq && !dq && (i + 1 == t.size() || std::isspace((unsigned char)t[i + 1]))) {
            key = unquote(trim(t.substr(0, i)));
            val = trim(t.substr(i + 1));
            return true;
        }
    }
    return false;
}

struct Parser {
    std::vector<Line> lines;
    size_t pos = 0;

    // parse a block whose lines are indented exactly `indent`
    YNode block(int indent) {
        YNode n;
        if (pos >= lines.size() || lines[pos].indent < indent) return n;
        indent = lines[pos].indent;
        const bool is_seq = lines[pos].text.rfind("- ", 0) == 0 || lines[pos].text == "-";
        if (is_seq) {
            n.kind = YNode::Seq;
            while (pos < lines.size() && lines[pos].indent == indent &&
                   (lines[pos].text.rfind("- ", 0) == 0 || lines[pos].text == "-")) {
                std::string rest = lines[pos].text == "-" ? "" : trim(lines[pos].text.substr(2));
                const int item_indent = indent + 2 + (int)(lines[pos].text.size() - 2 - rest.size() - 0);
                if (rest.empty()) {
                    ++pos;
                    n.seq.push_back(block(indent + 1));
                    continue;
                }
                // the item's first line is rewritten in place as a line of its own
                lines[pos].indent = indent + 2;
                lines[pos].text = rest;
                (void)item_indent;
                n.seq.push_back(block(indent + 2));
            }
            return n;
        }
        std::string key, val;
        if (!split_kv(lines[pos].text, key, val)) {
            // plain scalar
            n.kind = YNode::Scalar;
            n.scalar = unquote(lines[pos].text);
            ++pos;
            return n;
        }
        n.kind = YNode::Map;
        while (pos < lines.size() && lines[pos].indent == indent) {
            if (!split_kv(lines[pos].text, key, val))
                throw ConfigurationError("YAML: expected 'key: value' at \"" + lines[pos].text + "\"");
            ++pos;
            YNode child;
            if (!val.empty()) {
                child.kind = YNode::Scalar;
                child.scalar = unquote(val);
            } else if (pos < lines.size() && lines[pos].indent > indent) {
                child = block(indent + 1);
            } else if (pos < lines.size() && lines[pos].indent == indent &&
                       (lines[pos].text.rfind("- ", 0) == 0 || lines[pos].text == "-")) {
                // sequence at the same indentation as its key (allowed in YAML)
                child = block(indent);
            }
            n.map.emplace_back(key, std::move(child));
        }
        return n;
    }
};
}  // namespace

YNode parse_yaml(const std::string& text) {
    Parser p;
    std::istringstream in(text);
    std::string raw;
    while (std::getline(in, raw)) {
        for (auto& c : raw)
            if (c == '\t') c = ' ';
        const std::string s = strip_comment(raw);
        const std::string t = trim(s);
        if (t.empty() || t == "---") continue;
        int ind = 0;
        while (ind < (int)s.size() && s[ind] == ' ') ++ind;
        p.lines.push_back({ind, t});
    }
    if (p.lines.empty()) return YNode();
    YNode root = p.block(p.lines[0].indent);
    if (p.pos != p.lines.size())
        throw ConfigurationError("YAML: unexpected indentation at \"" + p.lines[p.pos].text + "\"");
    return root;
}

}  // namespace pm
