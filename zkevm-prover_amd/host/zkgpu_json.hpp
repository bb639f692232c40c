// zkgpu_json.hpp -- the JSON the drop-in driver reads and writes.
//
// The reference reads its starkinfo / config / verkey files and writes its
// proofs with nlohmann::json (stark_info.cpp:13-17, utils.cpp:212-222
// json2file: `outputStream << setw(4) << j << endl`).  The image has no
// nlohmann, so this is a small parser plus a writer producing that exact
// layout: objects keep insertion order (ordered_json), numbers keep their
// literal text (u64 values are exact), dump4() = nlohmann's dump(4).
#pragma once
#include <ctype.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace zkgpu {
namespace json {

struct Value {
    enum Kind { Null, Bool, Number, String, Array, Object };
    Kind kind = Null;
    bool b = false;
    std::string s;  // String: the text; Number: the literal
    std::vector<Value> a;
    std::vector<std::pair<std::string, Value>> o;

    static Value str(std::string v)
    {
        Value r;
        r.kind = String;
        r.s = std::move(v);
        return r;
    }
    static Value num(uint64_t v)
    {
        Value r;
        r.kind = Number;
        r.s = std::to_string(v);
        return r;
    }
    static Value array()
    {
        Value r;
        r.kind = Array;
        return r;
    }
    static Value object()
    {
        Value r;
        r.kind = Object;
        return r;
    }

    bool is_null() const { return kind == Null; }
    size_t size() const { return kind == Array ? a.size() : kind == Object ? o.size() : 0; }
    bool contains(const std::string &k) const
    {
        if (kind != Object) return false;
        for (const auto &kv : o)
            if (kv.first == k) return true;
        return false;
    }
    const Value &operator[](const std::string &k) const
    {
        if (kind == Object)
            for (const auto &kv : o)
                if (kv.first == k) return kv.second;
        throw std::runtime_error("json: missing key \"" + k + "\"");
    }
    const Value &operator[](size_t i) const
    {
        if (kind != Array || i >= a.size()) throw std::runtime_error("json: index out of range");
        return a[i];
    }
    // object insertion (ordered_json semantics: an existing key keeps its place)
    Value &set(const std::string &k, Value v)
    {
        if (kind == Null) kind = Object;
        for (auto &kv : o)
            if (kv.first == k) return kv.second = std::move(v);
        o.emplace_back(k, std::move(v));
        return o.back().second;
    }
    void push(Value v)
    {
        if (kind == Null) kind = Array;
        a.push_back(std::move(v));
    }
    // unsigned integer (a number, or a string of decimal digits)
    uint64_t u64() const
    {
        if ((kind != Number && kind != String) || s.empty()) throw std::runtime_error("json: not an integer");
        uint64_t v = 0;
        for (char c : s) {
            if (c < '0' || c > '9') throw std::runtime_error("json: not an unsigned integer: " + s);
            const uint64_t d = (uint64_t)(c - '0');
            if (v > (UINT64_MAX - d) / 10) throw std::runtime_error("json: integer overflow: " + s);
            v = v * 10 + d;
        }
        return v;
    }
    bool boolean() const
    {
        if (kind == Bool) return b;
        if (kind == Number) return u64() != 0;
        throw std::runtime_error("json: not a boolean");
    }
    const std::string &string() const
    {
        if (kind != String) throw std::runtime_error("json: not a string");
        return s;
    }
};

class Parser
{
public:
    explicit Parser(const std::string &t) : t_(t) {}
    Value parse()
    {
        Value v = value();
        ws();
        if (p_ != t_.size()) err("trailing characters");
        return v;
    }

private:
    const std::string &t_;
    size_t p_ = 0;

    [[noreturn]] void err(const char *what) const
    {
        throw std::runtime_error(std::string("json: ") + what + " at offset " + std::to_string(p_));
    }
    void ws()
    {
        while (p_ < t_.size() && (t_[p_] == ' ' || t_[p_] == '\n' || t_[p_] == '\r' || t_[p_] == '\t')) p_++;
    }
    bool lit(const char *w)
    {
        size_t n = 0;
        while (w[n]) n++;
        if (t_.compare(p_, n, w) == 0) {
            p_ += n;
            return true;
        }
        return false;
    }
    std::string string_body()
    {
        if (t_[p_] != '"') err("expected string");
        p_++;
        std::string out;
        while (p_ < t_.size() && t_[p_] != '"') {
            char c = t_[p_++];
            if (c == '\\') {
                if (p_ >= t_.size()) err("bad escape");
                const char e = t_[p_++];
                switch (e) {
                case '"': out += '"'; break;
                case '\\': out += '\\'; break;
                case '/': out += '/'; break;
                case 'b': out += '\b'; break;
                case 'f': out += '\f'; break;
                case 'n': out += '\n'; break;
                case 'r': out += '\r'; break;
                case 't': out += '\t'; break;
                case 'u': {
                    if (p_ + 4 > t_.size()) err("bad \\u escape");
                    const unsigned cp = (unsigned)strtoul(t_.substr(p_, 4).c_str(), nullptr, 16);
                    p_ += 4;
                    if (cp < 0x80) out += (char)cp;
                    else if (cp < 0x800) {
                        out += (char)(0xC0 | (cp >> 6));
                        out += (char)(0x80 | (cp & 0x3F));
                    } else {
                        out += (char)(0xE0 | (cp >> 12));
                        out += (char)(0x80 | ((cp >> 6) & 0x3F));
                        out += (char)(0x80 | (cp & 0x3F));
                    }
                    break;
                }
                default: err("bad escape");
                }
            } else {
                out += c;
            }
        }
        if (p_ >= t_.size()) err("unterminated string");
        p_++;
        return out;
    }
    Value value()
    {
        ws();
        if (p_ >= t_.size()) err("unexpected end");
        const char c = t_[p_];
        Value v;
        if (c == '{') {
            p_++;
            v.kind = Value::Object;
            ws();
            if (p_ < t_.size() && t_[p_] == '}') {
                p_++;
                return v;
            }
            for (;;) {
                ws();
                std::string k = string_body();
                ws();
                if (p_ >= t_.size() || t_[p_] != ':') err("expected ':'");
                p_++;
                v.o.emplace_back(std::move(k), value());
                ws();
                if (p_ < t_.size() && t_[p_] == ',') {
                    p_++;
                    continue;
                }
                if (p_ < t_.size() && t_[p_] == '}') {
                    p_++;
                    return v;
                }
                err("expected ',' or '}'");
            }
        }
        if (c == '[') {
            p_++;
            v.kind = Value::Array;
            ws();
            if (p_ < t_.size() && t_[p_] == ']') {
                p_++;
                return v;
            }
            for (;;) {
                v.a.push_back(value());
                ws();
                if (p_ < t_.size() && t_[p_] == ',') {
                    p_++;
                    continue;
                }
                if (p_ < t_.size() && t_[p_] == ']') {
                    p_++;
                    return v;
                }
                err("expected ',' or ']'");
            }
        }
        if (c == '"') {
            v.kind = Value::String;
            v.s = string_body();
            return v;
        }
        if (lit("true")) {
            v.kind = Value::Bool;
            v.b = true;
            return v;
        }
        if (lit("false")) {
            v.kind = Value::Bool;
            return v;
        }
        if (lit("null")) return v;
        if (c == '-' || (c >= '0' && c <= '9')) {
            const size_t s0 = p_;
            p_++;
            while (p_ < t_.size() && (isdigit((unsigned char)t_[p_]) || t_[p_] == '.' || t_[p_] == 'e' ||
                                      t_[p_] == 'E' || t_[p_] == '+' || t_[p_] == '-'))
                p_++;
            v.kind = Value::Number;
            v.s = t_.substr(s0, p_ - s0);
            return v;
        }
        err("unexpected character");
    }
};

inline Value parse(const std::string &text) { return Parser(text).parse(); }

inline void dump_rec(const Value &v, std::string &out, int level)
{
    auto ind = [&](int l) { out.append((size_t)(4 * l), ' '); };
    switch (v.kind) {
    case Value::Null: out += "null"; break;
    case Value::Bool: out += v.b ? "true" : "false"; break;
    case Value::Number: out += v.s; break;
    case Value::String: {
        out += '"';
        for (char c : v.s) {
            switch (c) {
            case '"': out += "\\\""; break;
            case '\\': out += "\\\\"; break;
            case '\n': out += "\\n"; break;
            case '\t': out += "\\t"; break;
            case '\r': out += "\\r"; break;
            case '\b': out += "\\b"; break;
            case '\f': out += "\\f"; break;
            default:
                if ((unsigned char)c < 0x20) {
                    char buf[8];
                    snprintf(buf, sizeof buf, "\\u%04x", (unsigned char)c);
                    out += buf;
                } else {
                    out += c;
                }
            }
        }
        out += '"';
        break;
    }
    case Value::Array:
        if (v.a.empty()) {
            out += "[]";
            break;
        }
        out += "[\n";
        for (size_t i = 0; i < v.a.size(); i++) {
            ind(level + 1);
            dump_rec(v.a[i], out, level + 1);
            out += i + 1 < v.a.size() ? ",\n" : "\n";
        }
        ind(level);
        out += ']';
        break;
    case Value::Object:
        if (v.o.empty()) {
            out += "{}";
            break;
        }
        out += "{\n";
        for (size_t i = 0; i < v.o.size(); i++) {
            ind(level + 1);
            dump_rec(Value::str(v.o[i].first), out, level + 1);
            out += ": ";
            dump_rec(v.o[i].second, out, level + 1);
            out += i + 1 < v.o.size() ? ",\n" : "\n";
        }
        ind(level);
        out += '}';
        break;
    }
}

// nlohmann dump(4) (json2file adds the trailing newline)
inline std::string dump4(const Value &v)
{
    std::string out;
    dump_rec(v, out, 0);
    return out;
}

}  // namespace json
}  // namespace zkgpu
