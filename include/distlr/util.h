// distlr/util.h -- drop-in for the reference's include/util.h.
// Same declarations (include/util.h:9-17); implemented over the C-ABI
// (dlr_split / dlr_to_int / dlr_to_float) with src/util.cc's semantics,
// quirks included (see DESIGN.md "Parsing").
#ifndef DISTLR_AMD_UTIL_H_
#define DISTLR_AMD_UTIL_H_

#include <string>
#include <vector>

namespace distlr {

std::vector<std::string> Split(std::string line, char separator);

int ToInt(const char *str);

int ToInt(const std::string &str);

float ToFloat(const char *str);

float ToFloat(const std::string &str);

}  // namespace distlr

#endif  // DISTLR_AMD_UTIL_H_
