// N-Queens device engine factory (definitions in queens_engine.hip).
#pragma once

#include <memory>
#include <vector>

#include "engine.hpp"
#include "../core/pfsp_node.hpp"

namespace tts {

std::unique_ptr<IEngine> make_queens_engine(int N, int G, const EngineConfig& cfg);
std::vector<uint8_t> queens_gpu_labels(int N, int G, const QueensNode* parents, size_t n, int device);

}  // namespace tts
