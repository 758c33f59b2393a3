// FrodoKEM-640/976-SHAKE batched KeyGen / Encaps / Decaps (placeholder: the
// HIP implementation is added in a later commit; until then the weak stubs in
// util.hip report hipErrorNotSupported and the algorithms are not enabled).
#include "qrkem_internal.h"
