// Definitions shared by the C-ABI translation units (not part of the ABI).
#pragma once
#include <memory>

#include "scanner.h"

struct tsg_scanner {
  std::unique_ptr<tsg::SecretScanner> s;
};
