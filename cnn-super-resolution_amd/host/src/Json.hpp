// Minimal JSON reader/writer for config.json and parameters.json.
//
// The reference parses with the vendored gason library
// (src/pch.cpp read_json_file / try_read_*); this is an independent
// recursive-descent parser with the same observable contract: object keys
// keep file order, numbers are doubles, a syntax error or a missing file
// throws IOException, a wrong root type throws std::runtime_error.
#ifndef SRCNN_HOST_JSON_HPP
#define SRCNN_HOST_JSON_HPP

#include <string>
#include <utility>
#include <vector>

namespace srcnn {
namespace json {

enum class Tag { Number, String, Array, Object, True, False, Null };

struct Value {
  Tag tag = Tag::Null;
  double number = 0.0;
  std::string string;
  std::vector<Value> array;
  std::vector<std::pair<std::string, Value>> object;

  bool is(Tag t) const { return tag == t; }
  /** member `key` of an object, or nullptr */
  const Value* find(const std::string& key) const;
};

/** Parse a whole document (throws IOException on a syntax error). */
Value parse(const std::string& text);

/** Read + parse a file; `root` is the required root tag (reference
 * read_json_file: IOException for I/O and syntax, runtime_error for root). */
Value parse_file(const std::string& path, Tag root = Tag::Object);

/** try_read_* of the reference (src/pch.cpp): assign when `key` matches and
 * the value has the expected type. */
bool try_read_float(const std::string& key, const Value& v, float& lhs, const char* want);
bool try_read_uint(const std::string& key, const Value& v, size_t& lhs, const char* want);
bool try_read_string(const std::string& key, const Value& v, std::string& lhs, const char* want);
bool try_read_vector(const std::string& key, const Value& v, std::vector<float>& lhs,
                     const char* want);

/** Shortest decimal text that reads back to exactly `x` (lossless floats). */
std::string format_float(float x);

}  // namespace json
}  // namespace srcnn

#endif  // SRCNN_HOST_JSON_HPP
