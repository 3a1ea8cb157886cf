// plugin_latency.hpp -- the config-1 plugin path timed from C++ (see
// plugin_latency.cpp): median milliseconds per named step.
#pragma once

#include <map>
#include <string>
#include <vector>

#include "infectious.hpp"

namespace rsmi_host {

Status PluginLatency(const std::vector<uint8_t>& blob, int k, int n, const std::vector<int>& dropped, int reps,
                     std::map<std::string, double>* out);

}  // namespace rsmi_host
