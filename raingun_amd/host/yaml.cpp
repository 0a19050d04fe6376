// yaml.cpp — see yaml.h.  A recursive-descent parser over block/flow YAML that
// builds a Node tree; scalar typing is deferred to resolve(), which follows
// yaml-rust 0.3.5's Yaml::from_str (plain scalars only; quoted scalars are
// always strings).
#include "yaml.h"

#include <cerrno>
#include <cmath>
#include <cstdlib>
#include <limits>
#include <map>

namespace rgh {
namespace yaml {

const Node *Node::get(const std::string &key) const {
    for (const auto &kv : map)
        if (kv.first == key) return &kv.second;
    return nullptr;
}

// ---------------------------------------------------------------- resolution
bool rust_parse_i64(const std::string &s, int64_t *out) {
    size_t i = 0;
    bool neg = false;
    if (i < s.size() && (s[i] == '+' || s[i] == '-')) { neg = s[i] == '-'; ++i; }
    if (i == s.size()) return false;
    uint64_t v = 0;
    const uint64_t lim = neg ? (uint64_t)std::numeric_limits<int64_t>::max() + 1 : (uint64_t)std::numeric_limits<int64_t>::max();
    for (; i < s.size(); ++i) {
        if (s[i] < '0' || s[i] > '9') return false;
        uint64_t d = (uint64_t)(s[i] - '0');
        if (v > (lim - d) / 10) return false;
        v = v * 10 + d;
    }
    if (out) *out = neg ? (int64_t)(0 - v) : (int64_t)v;
    return true;
}

static bool parse_radix_i64(const std::string &s, int radix, int64_t *out) {
    // i64::from_str_radix: optional sign, then at least one digit of `radix`
    size_t i = 0;
    bool neg = false;
    if (i < s.size() && (s[i] == '+' || s[i] == '-')) { neg = s[i] == '-'; ++i; }
    if (i == s.size()) return false;
    __int128 v = 0;
    for (; i < s.size(); ++i) {
        int c = s[i], d;
        if (c >= '0' && c <= '9') d = c - '0';
        else if (c >= 'a' && c <= 'z') d = c - 'a' + 10;
        else if (c >= 'A' && c <= 'Z') d = c - 'A' + 10;
        else return false;
        if (d >= radix) return false;
        v = v * radix + d;
        if (v > (__int128)std::numeric_limits<int64_t>::max() + 1) return false;
    }
    if (neg) v = -v;
    if (v > std::numeric_limits<int64_t>::max() || v < std::numeric_limits<int64_t>::min()) return false;
    if (out) *out = (int64_t)v;
    return true;
}

bool rust_parse_f64(const std::string &s, double *out) {
    size_t i = 0;
    bool neg = false;
    if (i < s.size() && (s[i] == '+' || s[i] == '-')) { neg = s[i] == '-'; ++i; }
    const std::string rest = s.substr(i);
    if (rest == "inf") { if (out) *out = neg ? -HUGE_VAL : HUGE_VAL; return true; }
    if (rest == "NaN") { if (out) *out = std::nan(""); return true; }
    size_t d1 = 0, d2 = 0;
    while (i < s.size() && s[i] >= '0' && s[i] <= '9') { ++i; ++d1; }
    if (i < s.size() && s[i] == '.') {
        ++i;
        while (i < s.size() && s[i] >= '0' && s[i] <= '9') { ++i; ++d2; }
    }
    if (d1 + d2 == 0) return false;
    if (i < s.size() && (s[i] == 'e' || s[i] == 'E')) {
        ++i;
        if (i < s.size() && (s[i] == '+' || s[i] == '-')) ++i;
        size_t d3 = 0;
        while (i < s.size() && s[i] >= '0' && s[i] <= '9') { ++i; ++d3; }
        if (d3 == 0) return false;
    }
    if (i != s.size()) return false;
    if (out) {
        errno = 0;
        *out = std::strtod(s.c_str(), nullptr);  // correctly rounded (glibc), like dec2flt
    }
    return true;
}

ScalarType resolve(const Node &n, int64_t *ival, double *rval, bool *bval) {
    if (n.kind == Node::Null) return ScalarType::Null;
    if (n.kind != Node::Scalar) return ScalarType::String;  // caller checks kind first
    if (!n.plain) return ScalarType::String;
    const std::string &v = n.str;
    int64_t i = 0;
    if (v.compare(0, 2, "0x") == 0 && parse_radix_i64(v.substr(2), 16, &i)) { if (ival) *ival = i; return ScalarType::Integer; }
    if (v.compare(0, 2, "0o") == 0 && parse_radix_i64(v.substr(2), 8, &i)) { if (ival) *ival = i; return ScalarType::Integer; }
    if (!v.empty() && v[0] == '+' && rust_parse_i64(v.substr(1), &i)) { if (ival) *ival = i; return ScalarType::Integer; }
    if (v == "~" || v == "null") return ScalarType::Null;
    if (v == "true" || v == "false") { if (bval) *bval = v == "true"; return ScalarType::Bool; }
    if (rust_parse_i64(v, &i)) { if (ival) *ival = i; return ScalarType::Integer; }
    double d;
    if (rust_parse_f64(v, &d)) { if (rval) *rval = d; return ScalarType::Real; }
    return ScalarType::String;
}

// ---------------------------------------------------------------- parser
namespace {

struct Error {
    std::string msg;
    int line, col;
};

inline bool is_blank(char c) { return c == ' ' || c == '\t'; }
inline bool is_flow_ind(char c) { return c == ',' || c == '[' || c == ']' || c == '{' || c == '}'; }

void append_utf8(std::string &o, uint32_t cp) {
    if (cp < 0x80) o += (char)cp;
    else if (cp < 0x800) { o += (char)(0xC0 | (cp >> 6)); o += (char)(0x80 | (cp & 63)); }
    else if (cp < 0x10000) { o += (char)(0xE0 | (cp >> 12)); o += (char)(0x80 | ((cp >> 6) & 63)); o += (char)(0x80 | (cp & 63)); }
    else { o += (char)(0xF0 | (cp >> 18)); o += (char)(0x80 | ((cp >> 12) & 63)); o += (char)(0x80 | ((cp >> 6) & 63)); o += (char)(0x80 | (cp & 63)); }
}

struct Parser {
    std::string s;
    size_t pos = 0, line_start = 0;
    int line = 1;
    std::map<std::string, Node> anchors;

    explicit Parser(const std::string &text) {
        s.reserve(text.size());
        for (size_t i = 0; i < text.size(); ++i) {  // normalise line breaks
            if (text[i] == '\r') { s += '\n'; if (i + 1 < text.size() && text[i + 1] == '\n') ++i; }
            else s += text[i];
        }
        if (s.size() >= 3 && (unsigned char)s[0] == 0xEF && (unsigned char)s[1] == 0xBB && (unsigned char)s[2] == 0xBF)
            s.erase(0, 3);  // BOM
    }
    int col() const { return (int)(pos - line_start); }
    char peek(size_t k = 0) const { return pos + k < s.size() ? s[pos + k] : '\0'; }
    bool eof() const { return pos >= s.size(); }
    bool blank_or_end(size_t k) const { char c = peek(k); return c == '\0' || c == ' ' || c == '\t' || c == '\n'; }
    void advance() {
        if (s[pos] == '\n') { ++line; line_start = pos + 1; }
        ++pos;
    }
    [[noreturn]] void fail(const std::string &m) { throw Error{m, line, col() + 1}; }

    void skip_inline_ws() { while (is_blank(peek())) advance(); }
    void skip_comment() { if (peek() == '#') while (!eof() && peek() != '\n') advance(); }
    bool at_line_end() {
        skip_inline_ws();
        return eof() || peek() == '\n' || peek() == '#';
    }
    void expect_line_end() {
        if (!at_line_end()) fail("unexpected content after a value");
        skip_comment();
    }
    // Skip blanks, comments and line breaks up to the next content character.
    void skip_to_content() {
        for (;;) {
            bool leading = pos == line_start;
            while (is_blank(peek())) {
                if (leading && peek() == '\t') {
                    size_t q = pos;
                    while (q < s.size() && is_blank(s[q])) ++q;
                    if (q < s.size() && s[q] != '\n' && s[q] != '#') fail("tabs are not allowed as indentation");
                }
                advance();
            }
            if (peek() == '#') skip_comment();
            if (peek() == '\n') { advance(); continue; }
            return;
        }
    }
    bool at_doc_marker() const {
        if (col() != 0 || pos + 3 > s.size()) return false;
        if (s.compare(pos, 3, "---") != 0 && s.compare(pos, 3, "...") != 0) return false;
        char c = pos + 3 < s.size() ? s[pos + 3] : '\0';
        return c == '\0' || c == ' ' || c == '\t' || c == '\n';
    }

    static void set(Node &m, const std::string &k, Node v) {
        for (auto &kv : m.map)
            if (kv.first == k) { kv.second = std::move(v); return; }
        m.map.emplace_back(k, std::move(v));
    }

    std::string read_name() {  // anchor / alias name
        size_t st = pos;
        while (!eof() && !is_blank(peek()) && peek() != '\n' && !is_flow_ind(peek())) advance();
        if (pos == st) fail("empty anchor or alias name");
        return s.substr(st, pos - st);
    }
    Node alias() {
        advance();  // '*'
        std::string n = read_name();
        auto it = anchors.find(n);
        if (it == anchors.end()) fail("unknown anchor '" + n + "'");
        return it->second;
    }

    // ---- scalars
    void fold_break(std::string &o) {
        // at '\n' inside a quoted scalar: trailing blanks already in `o` are trimmed;
        // one break folds to a space, n breaks to n-1 newlines
        while (!o.empty() && is_blank(o.back())) o.pop_back();
        int breaks = 0;
        while (peek() == '\n') {
            ++breaks;
            advance();
            while (is_blank(peek())) advance();
        }
        if (breaks == 1) o += ' ';
        else o.append((size_t)(breaks - 1), '\n');
    }
    Node single_quoted() {
        Node n;
        n.kind = Node::Scalar;
        n.line = line;
        advance();
        for (;;) {
            if (eof()) fail("unterminated single-quoted scalar");
            char c = peek();
            if (c == '\'') {
                if (peek(1) == '\'') { n.str += '\''; advance(); advance(); continue; }
                advance();
                break;
            }
            if (c == '\n') { fold_break(n.str); continue; }
            n.str += c;
            advance();
        }
        return n;
    }
    uint32_t hex(int digits) {
        uint32_t v = 0;
        for (int i = 0; i < digits; ++i) {
            char c = peek();
            int d = (c >= '0' && c <= '9') ? c - '0' : (c >= 'a' && c <= 'f') ? c - 'a' + 10 : (c >= 'A' && c <= 'F') ? c - 'A' + 10 : -1;
            if (d < 0) fail("bad hex escape");
            v = v * 16 + (uint32_t)d;
            advance();
        }
        return v;
    }
    Node double_quoted() {
        Node n;
        n.kind = Node::Scalar;
        n.line = line;
        advance();
        for (;;) {
            if (eof()) fail("unterminated double-quoted scalar");
            char c = peek();
            if (c == '"') { advance(); break; }
            if (c == '\n') { fold_break(n.str); continue; }
            if (c != '\\') { n.str += c; advance(); continue; }
            advance();
            char e = peek();
            if (e == '\n') {  // escaped line break: join without a space
                advance();
                while (is_blank(peek())) advance();
                continue;
            }
            advance();
            switch (e) {
            case '0': n.str += '\0'; break;
            case 'a': n.str += '\a'; break;
            case 'b': n.str += '\b'; break;
            case 't': case '\t': n.str += '\t'; break;
            case 'n': n.str += '\n'; break;
            case 'v': n.str += '\v'; break;
            case 'f': n.str += '\f'; break;
            case 'r': n.str += '\r'; break;
            case 'e': n.str += '\x1b'; break;
            case ' ': n.str += ' '; break;
            case '"': n.str += '"'; break;
            case '/': n.str += '/'; break;
            case '\\': n.str += '\\'; break;
            case 'N': append_utf8(n.str, 0x85); break;
            case '_': append_utf8(n.str, 0xA0); break;
            case 'L': append_utf8(n.str, 0x2028); break;
            case 'P': append_utf8(n.str, 0x2029); break;
            case 'x': append_utf8(n.str, hex(2)); break;
            case 'u': append_utf8(n.str, hex(4)); break;
            case 'U': append_utf8(n.str, hex(8)); break;
            default: fail(std::string("unknown escape '\\") + e + "'");
            }
        }
        return n;
    }
    Node plain(bool flow) {
        Node n;
        n.kind = Node::Scalar;
        n.plain = true;
        n.line = line;
        char c0 = peek();
        if (c0 == ',' || c0 == ']' || c0 == '}' || c0 == '@' || c0 == '`' || c0 == '!' || c0 == '%' ||
            (c0 == '?' && blank_or_end(1)))
            fail(std::string("unexpected character '") + c0 + "'" + (c0 == '!' ? " (tags are not supported)" : ""));
        size_t st = pos;
        while (!eof()) {
            char c = peek();
            if (c == '\n') break;
            if (c == ':' && (blank_or_end(1) || (flow && is_flow_ind(peek(1))))) break;
            if (c == '#' && pos > st && is_blank(s[pos - 1])) break;
            if (flow && is_flow_ind(c)) break;
            advance();
        }
        size_t e = pos;
        while (e > st && is_blank(s[e - 1])) --e;
        n.str = s.substr(st, e - st);
        if (n.str.empty()) n.kind = Node::Null;
        return n;
    }
    Node block_scalar(int parent_indent) {
        Node n;
        n.kind = Node::Scalar;
        n.line = line;
        const bool literal = peek() == '|';
        advance();
        int chomp = 0, explicit_indent = 0;  // chomp: 0 clip, -1 strip, +1 keep
        for (int k = 0; k < 2; ++k) {
            if (peek() == '-' || peek() == '+') { chomp = peek() == '-' ? -1 : 1; advance(); }
            else if (peek() >= '1' && peek() <= '9') { explicit_indent = peek() - '0'; advance(); }
        }
        if (!at_line_end()) fail("unexpected content after a block scalar indicator");
        skip_comment();
        if (peek() == '\n') advance();
        int indent = explicit_indent ? (parent_indent < 0 ? 0 : parent_indent) + explicit_indent : -1;
        std::vector<std::string> lines;
        for (;;) {
            if (eof()) break;
            size_t q = pos;
            int sp = 0;
            while (q < s.size() && s[q] == ' ') { ++q; ++sp; }
            bool empty = q >= s.size() || s[q] == '\n';
            if (!empty) {
                if (indent < 0) {
                    if (sp <= parent_indent) break;
                    indent = sp;
                }
                if (sp < indent) break;
            }
            size_t le = s.find('\n', pos);
            if (le == std::string::npos) le = s.size();
            std::string ln = s.substr(pos, le - pos);
            lines.push_back(indent >= 0 && (int)ln.size() >= indent ? ln.substr((size_t)indent) : (empty ? "" : ln));
            while (pos < le) advance();
            if (!eof()) advance();
        }
        size_t last = lines.size();
        while (last > 0 && lines[last - 1].find_first_not_of(' ') == std::string::npos) --last;
        std::string body;
        for (size_t i = 0; i < last; ++i) {
            const std::string &ln = lines[i];
            if (i > 0) {
                const std::string &prev = lines[i - 1];
                bool fold = !literal && !prev.empty() && !ln.empty() && prev[0] != ' ' && ln[0] != ' ';
                body += fold ? ' ' : '\n';
            }
            body += ln;
        }
        if (chomp == 1) {
            body += '\n';
            for (size_t i = last; i < lines.size(); ++i) body += '\n';
        } else if (chomp == 0 && last > 0) {
            body += '\n';
        }
        n.str = body;
        return n;
    }

    // ---- flow collections
    void skip_flow_ws() {
        for (;;) {
            while (is_blank(peek()) || peek() == '\n') advance();
            if (peek() == '#') { skip_comment(); continue; }
            return;
        }
    }
    Node flow_node() {
        std::string anchor;
        if (peek() == '&') {
            advance();
            anchor = read_name();
            skip_flow_ws();
        }
        Node n;
        char c = peek();
        if (c == '*') n = alias();
        else if (c == '[' || c == '{') n = flow();
        else if (c == '\'') n = single_quoted();
        else if (c == '"') n = double_quoted();
        else n = plain(true);
        if (!anchor.empty()) anchors[anchor] = n;
        return n;
    }
    std::string key_of(const Node &k) {
        if (k.kind != Node::Scalar) fail("only scalar mapping keys are supported");
        return k.str;
    }
    Node flow() {
        const char open = peek(), close = open == '[' ? ']' : '}';
        Node n;
        n.kind = open == '[' ? Node::Seq : Node::Map;
        n.line = line;
        advance();
        for (;;) {
            skip_flow_ws();
            if (eof()) fail("unterminated flow collection");
            if (peek() == close) { advance(); break; }
            Node item = flow_node();
            skip_flow_ws();
            bool pair = peek() == ':';
            Node value;
            if (pair) {
                advance();
                skip_flow_ws();
                if (peek() != ',' && peek() != close) value = flow_node();
            }
            if (n.kind == Node::Seq) {
                if (pair) {
                    Node m;
                    m.kind = Node::Map;
                    m.line = item.line;
                    set(m, key_of(item), std::move(value));
                    n.seq.push_back(std::move(m));
                } else {
                    n.seq.push_back(std::move(item));
                }
            } else {
                set(n, key_of(item), std::move(value));
            }
            skip_flow_ws();
            if (peek() == ',') advance();
            else if (peek() != close) fail(std::string("expected ',' or '") + close + "' in a flow collection");
        }
        return n;
    }

    // ---- block structure
    Node block_seq(int indent) {
        Node q;
        q.kind = Node::Seq;
        q.line = line;
        for (;;) {
            advance();  // '-'
            Node item;
            if (at_line_end()) {
                skip_to_content();
                if (!eof() && !at_doc_marker() && col() > indent) item = block_node(indent);
            } else {
                item = block_node(indent);
            }
            q.seq.push_back(std::move(item));
            skip_to_content();
            if (eof() || at_doc_marker() || col() < indent) break;
            if (col() > indent) fail("bad indentation of a sequence entry");
            if (!(peek() == '-' && blank_or_end(1))) break;
        }
        return q;
    }
    Node map_value(int indent) {
        std::string anchor;
        if (!at_line_end() && peek() == '&') {
            advance();
            anchor = read_name();
        }
        Node v;
        if (at_line_end()) {
            skip_to_content();
            if (!eof() && !at_doc_marker()) {
                if (col() > indent) v = block_node(indent);
                else if (col() == indent && peek() == '-' && blank_or_end(1)) v = block_seq(indent);
            }
        } else {
            char c = peek();
            if (c == '-' && blank_or_end(1)) fail("block sequence entries are not allowed in this context");
            if (c == '|' || c == '>') {
                v = block_scalar(indent);
            } else {
                if (c == '[' || c == '{') v = flow();
                else if (c == '*') v = alias();
                else if (c == '\'') v = single_quoted();
                else if (c == '"') v = double_quoted();
                else v = plain(false);
                skip_inline_ws();
                if (peek() == ':' && blank_or_end(1)) fail("mapping values are not allowed in this context");
                expect_line_end();
            }
        }
        if (!anchor.empty()) anchors[anchor] = v;
        return v;
    }
    Node block_map(int indent, std::string key, int key_line) {
        Node m;
        m.kind = Node::Map;
        m.line = key_line;
        for (;;) {
            advance();  // ':'
            Node v = map_value(indent);
            set(m, key, std::move(v));
            skip_to_content();
            if (eof() || at_doc_marker() || col() < indent) break;
            if (col() > indent) fail("bad indentation of a mapping entry");
            char c = peek();
            Node k;
            if (c == '\'') k = single_quoted();
            else if (c == '"') k = double_quoted();
            else if (c == '-' && blank_or_end(1)) fail("expected a mapping key, found a sequence entry");
            else if (c == '[' || c == '{' || c == '*' || c == '&' || (c == '?' && blank_or_end(1)))
                fail("only plain or quoted scalar mapping keys are supported");
            else k = plain(false);
            skip_inline_ws();
            if (!(peek() == ':' && blank_or_end(1))) fail("could not find expected ':'");
            key = key_of(k.kind == Node::Null ? fail_empty_key() : k);
        }
        return m;
    }
    [[noreturn]] Node fail_empty_key() { fail("empty mapping key"); }

    // A node starting at the current content position; structures it opens are
    // indented at the current column, which must be > parent_indent.
    Node block_node(int parent_indent) {
        if (col() <= parent_indent) fail("bad indentation");
        std::string anchor;
        if (peek() == '&') {
            advance();
            anchor = read_name();
            if (at_line_end()) {
                skip_to_content();
                Node n;
                if (!eof() && !at_doc_marker() && col() > parent_indent) n = block_node(parent_indent);
                anchors[anchor] = n;
                return n;
            }
        }
        Node n;
        const int c0 = col();
        const int l0 = line;
        char c = peek();
        if (c == '-' && blank_or_end(1)) {
            n = block_seq(c0);
        } else if (c == '|' || c == '>') {
            n = block_scalar(parent_indent);
        } else if (c == '[' || c == '{' || c == '*') {
            n = c == '*' ? alias() : flow();
            skip_inline_ws();
            if (peek() == ':' && blank_or_end(1)) fail("only plain or quoted scalar mapping keys are supported");
            expect_line_end();
        } else {
            Node k = c == '\'' ? single_quoted() : c == '"' ? double_quoted() : plain(false);
            skip_inline_ws();
            if (peek() == ':' && blank_or_end(1)) {
                if (k.kind == Node::Null) fail("empty mapping key");
                n = block_map(c0, k.str, l0);
            } else {
                expect_line_end();
                n = std::move(k);
            }
        }
        if (!anchor.empty()) anchors[anchor] = n;
        return n;
    }

    Node document() {
        skip_to_content();
        while (!eof() && col() == 0 && peek() == '%') {  // directives
            skip_comment();
            while (!eof() && peek() != '\n') advance();
            skip_to_content();
        }
        if (at_doc_marker() && s.compare(pos, 3, "---") == 0) {
            for (int i = 0; i < 3; ++i) advance();
            skip_to_content();
        }
        if (eof() || at_doc_marker()) return Node();
        Node n = block_node(-1);
        skip_to_content();
        if (!eof() && !at_doc_marker()) fail("unexpected content at the end of the document");
        return n;
    }
};

}  // namespace

bool parse(const std::string &text, Node &out, std::string &err) {
    Parser p(text);
    try {
        out = p.document();
        return true;
    } catch (const Error &e) {
        err = e.msg + " at line " + std::to_string(e.line) + " column " + std::to_string(e.col);
        return false;
    }
}

}  // namespace yaml
}  // namespace rgh
