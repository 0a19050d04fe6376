// yaml.h — the YAML subset scene files use, resolved the way the reference's
// yaml-rust 0.3.5 / serde_yaml 0.6.2 (Cargo.lock:883-890, 1155) resolve it.
//
// Supported: block mappings and sequences (including "- key: v" compact
// mappings and sequences at their parent key's indentation), flow "[...]" and
// "{...}" collections over several lines, plain / single-quoted /
// double-quoted scalars, literal "|" and folded ">" block scalars, anchors
// "&a" and aliases "*a", comments, "---" / "..." document markers (the first
// document is used).  Not supported (rejected with an error, never
// mis-parsed): tags, complex "? key" entries, multi-line plain scalars.
#pragma once
#include <cstdint>
#include <string>
#include <utility>
#include <vector>

namespace rgh {
namespace yaml {

struct Node {
    enum Kind { Null, Scalar, Seq, Map };
    Kind kind = Null;
    std::string str;   // scalar text (after unescaping)
    bool plain = false;  // plain scalar: subject to yaml-rust type resolution
    std::vector<Node> seq;
    std::vector<std::pair<std::string, Node>> map;  // insertion order; a repeated key overwrites
    int line = 0;      // 1-based source line

    const Node *get(const std::string &key) const;
};

// yaml-rust Yaml::from_str resolution of a plain scalar.
enum class ScalarType { Null, Bool, Integer, Real, String };
ScalarType resolve(const Node &n, int64_t *ival = nullptr, double *rval = nullptr, bool *bval = nullptr);

// Rust's `str::parse::<f64>` grammar (dec2flt): [+-]? (digits [. digits*] | . digits) ([eE][+-]?digits)?
// or [+-]?inf / [+-]?NaN.  Returns false when Rust would return Err.
bool rust_parse_f64(const std::string &s, double *out);
// Rust's `str::parse::<i64>`: [+-]?digits, in range.
bool rust_parse_i64(const std::string &s, int64_t *out);

bool parse(const std::string &text, Node &out, std::string &err);

}  // namespace yaml
}  // namespace rgh
