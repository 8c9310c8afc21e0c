// rt_build_id() (include/distraytracer.h, ABI 5): the hash distraytracer_old_amd/build.py computes over
// every source, header and flag of the library. It lives in this one translation unit so that a
// rebuild recompiles only the sources that changed (build.py caches the other objects by content).
#ifndef RT_BUILD_ID
#define RT_BUILD_ID "unknown"
#endif
extern "C" const char* rt_build_id(void) { return RT_BUILD_ID; }
