// Definitions shared by the C-ABI translation units (not part of the ABI).
#pragma once
#include <memory>
#include <string>
#include <vector>

#include "scanner.h"
#include "tsg_scanner.h"

struct tsg_scanner {
  std::unique_ptr<tsg::SecretScanner> s;
};

struct tsg_result {
  tsg::BatchResult files;
  tsg_stats stats;
  std::string json;        // tsg_result_json: every file (built once)
  std::string json_range;  // tsg_result_json_range: the last range asked for
  const tsg::SecretScanner* owner;
  std::unique_ptr<tsg::SecretScanner> owned;  // results of scanners made for one call (oracle hooks)
};

namespace tsg {
void SetError(const std::string& e);
// tsg_global -> the host scanner's rule specs (capi_scanner.cpp)
bool MakeRules(const tsg_global* g, std::vector<RuleSpec>* rules, std::string* err);
bool MakeAllow(const tsg_allow_rule* a, uint32_t n, std::vector<AllowRuleSpec>* out, std::string* err);
bool MakeExclude(const char* const* rx, uint32_t n, std::vector<std::unique_ptr<Regex>>* out, std::string* err);
}  // namespace tsg
