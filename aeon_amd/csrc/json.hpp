// json.hpp -- a small JSON reader for aeon's configuration objects (replaces the vendored
// nlohmann::json, src/json.hpp, for the few shapes aeon's configs use: objects, arrays,
// numbers, strings, booleans, null).
#pragma once
#include <cstdlib>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace aeon_hip {

class Json {
public:
    enum Type { NUL, BOOL, NUMBER, STRING, ARRAY, OBJECT };

    Json() = default;
    static Json parse(const std::string& text)
    {
        size_t i = 0;
        Json   v = parse_value(text, i, 0);
        skip_ws(text, i);
        if (i != text.size()) throw std::invalid_argument("json: trailing characters");
        return v;
    }

    Type               type() const { return m_type; }
    bool               is_null() const { return m_type == NUL; }
    bool               is_object() const { return m_type == OBJECT; }
    bool               is_array() const { return m_type == ARRAY; }
    bool               is_number() const { return m_type == NUMBER; }
    bool               is_string() const { return m_type == STRING; }
    bool               is_bool() const { return m_type == BOOL; }
    double             number() const { return expect(NUMBER, "number"), m_num; }
    bool               boolean() const { return expect(BOOL, "boolean"), m_bool; }
    const std::string& str() const { return expect(STRING, "string"), m_str; }
    const std::vector<Json>& array() const { return expect(ARRAY, "array"), m_arr; }
    const std::map<std::string, Json>& object() const { return expect(OBJECT, "object"), m_obj; }

    bool        has(const std::string& k) const { return m_type == OBJECT && m_obj.count(k) != 0; }
    const Json& at(const std::string& k) const
    {
        auto it = object().find(k);
        if (it == m_obj.end()) throw std::invalid_argument("json: missing key '" + k + "'");
        return it->second;
    }

private:
    Type                        m_type = NUL;
    bool                        m_bool = false;
    double                      m_num  = 0;
    std::string                 m_str;
    std::vector<Json>           m_arr;
    std::map<std::string, Json> m_obj;

    void expect(Type t, const char* what) const
    {
        if (m_type != t) throw std::invalid_argument(std::string("json: expected ") + what);
    }
    static void skip_ws(const std::string& s, size_t& i)
    {
        while (i < s.size() && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) i++;
    }
    static std::string parse_string(const std::string& s, size_t& i)
    {
        std::string out;
        i++; // opening quote
        while (i < s.size() && s[i] != '"') {
            char c = s[i++];
            if (c == '\\') {
                if (i >= s.size()) break;
                char e = s[i++];
                switch (e) {
                case 'n': out += '\n'; break;
                case 't': out += '\t'; break;
                case 'r': out += '\r'; break;
                case 'b': out += '\b'; break;
                case 'f': out += '\f'; break;
                case 'u': {
                    if (i + 4 > s.size()) throw std::invalid_argument("json: bad \\u escape");
                    unsigned cp = std::strtoul(s.substr(i, 4).c_str(), nullptr, 16);
                    i += 4;
                    if (cp < 0x80) out += (char)cp;
                    else if (cp < 0x800) out += (char)(0xC0 | (cp >> 6)), out += (char)(0x80 | (cp & 0x3F));
                    else
                        out += (char)(0xE0 | (cp >> 12)), out += (char)(0x80 | ((cp >> 6) & 0x3F)),
                            out += (char)(0x80 | (cp & 0x3F));
                    break;
                }
                default: out += e;
                }
            } else {
                out += c;
            }
        }
        if (i >= s.size()) throw std::invalid_argument("json: unterminated string");
        i++;
        return out;
    }
    // Nesting deeper than any configuration needs is refused (recursive descent: the untrusted text
    // must not be able to exhaust the stack).
    static constexpr int kMaxDepth = 256;
    static Json parse_value(const std::string& s, size_t& i, int depth)
    {
        if (depth > kMaxDepth) throw std::invalid_argument("json: nesting too deep");
        skip_ws(s, i);
        if (i >= s.size()) throw std::invalid_argument("json: unexpected end");
        Json v;
        char c = s[i];
        if (c == '{') {
            v.m_type = OBJECT;
            i++;
            skip_ws(s, i);
            if (i < s.size() && s[i] == '}') return i++, v;
            for (;;) {
                skip_ws(s, i);
                if (i >= s.size() || s[i] != '"') throw std::invalid_argument("json: expected key");
                std::string k = parse_string(s, i);
                skip_ws(s, i);
                if (i >= s.size() || s[i] != ':') throw std::invalid_argument("json: expected ':'");
                i++;
                v.m_obj[k] = parse_value(s, i, depth + 1);
                skip_ws(s, i);
                if (i < s.size() && s[i] == ',') { i++; continue; }
                if (i < s.size() && s[i] == '}') { i++; break; }
                throw std::invalid_argument("json: expected ',' or '}'");
            }
        } else if (c == '[') {
            v.m_type = ARRAY;
            i++;
            skip_ws(s, i);
            if (i < s.size() && s[i] == ']') return i++, v;
            for (;;) {
                v.m_arr.push_back(parse_value(s, i, depth + 1));
                skip_ws(s, i);
                if (i < s.size() && s[i] == ',') { i++; continue; }
                if (i < s.size() && s[i] == ']') { i++; break; }
                throw std::invalid_argument("json: expected ',' or ']'");
            }
        } else if (c == '"') {
            v.m_type = STRING;
            v.m_str  = parse_string(s, i);
        } else if (s.compare(i, 4, "true") == 0) {
            v.m_type = BOOL, v.m_bool = true, i += 4;
        } else if (s.compare(i, 5, "false") == 0) {
            v.m_type = BOOL, v.m_bool = false, i += 5;
        } else if (s.compare(i, 4, "null") == 0) {
            v.m_type = NUL, i += 4;
        } else {
            char*       end = nullptr;
            const char* b   = s.c_str() + i;
            v.m_num         = std::strtod(b, &end);
            if (end == b) throw std::invalid_argument("json: bad value");
            v.m_type = NUMBER;
            i += (size_t)(end - b);
        }
        return v;
    }
};

} // namespace aeon_hip
