// Kernel instantiations for the 500-job node bucket (one TU per bucket so the
// instantiations compile in parallel).
#include "pfsp_engine.hpp"

namespace tts {
TTS_PFSP_DEFINE_BUCKET(500)
}  // namespace tts
