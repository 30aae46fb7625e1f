// Kernel instantiations for the 200-job node bucket (one TU per bucket so the
// instantiations compile in parallel).
#include "pfsp_engine.hpp"

namespace tts {
TTS_PFSP_DEFINE_BUCKET(200)
}  // namespace tts
