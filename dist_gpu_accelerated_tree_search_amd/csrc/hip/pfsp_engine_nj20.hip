// Kernel instantiations for the 20-job node bucket (one TU per bucket so the
// instantiations compile in parallel).
#include "pfsp_engine.hpp"

namespace tts {
TTS_PFSP_DEFINE_BUCKET(20)
}  // namespace tts
