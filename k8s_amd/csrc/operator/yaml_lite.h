// A small YAML reader (block mappings/sequences, plain/quoted scalars, flow
// [..]/{..} collections, comments, `---`, `|`/`>` block scalars) producing
// Json. Enough for controller config files, TfJob manifests and kubeconfig.
// Scalars are typed like YAML 1.2 core: null/true/false/ints/floats, the rest
// strings.
#pragma once

#include <string>
#include <vector>

#include "json.h"

namespace tfop {

Json yaml_parse(const std::string& text);                  // first document
std::vector<Json> yaml_parse_all(const std::string& text);  // every `---` document
std::string read_file(const std::string& path);

}  // namespace tfop
