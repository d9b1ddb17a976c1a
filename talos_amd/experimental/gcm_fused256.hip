// gcm_fused256.hip — AES-256 instantiations of the fused kernel (see gcm_fused.hip).
#define TG_FUSED_ROUNDS 14
#include "gcm_fused.hip"
