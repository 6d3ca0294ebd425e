// acehip_build_hash(): the native-source hash this library was built from (csrc/native_hash.py,
// passed in by the Makefile); acehip/_ffi.py compares it with the tree it loads the library from.
#ifndef ACEHIP_BUILD_HASH
#error "ACEHIP_BUILD_HASH must be defined by the Makefile"
#endif
extern "C" const char *acehip_build_hash(void) { return ACEHIP_BUILD_HASH; }
