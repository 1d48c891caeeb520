// frames.h — internal interface between render.hip (the single-device
// context) and frames.hip (a context over several devices, the
// device-resident Image). Not part of the C ABI.
#pragma once
#include <stdint.h>

#include <string>

#include "../../../include/massrt.h"

struct MultiDev;  // frames.hip

// ---- frames.hip ----
int multi_count(const MultiDev* m);
mrt_ctx* multi_dev(const MultiDev* m, int i);  // the single-device context of device slot i
void multi_free(MultiDev* m);
// mrt_render on every device (host accumulation buffers); MRT_OK or a code + err
int multi_render(MultiDev* m, const mrt_render_args* a, float* rgb, uint32_t* bounces, std::string& err);
// option "gather" (MRT_GATHER_*): MRT_OK or a code + err; the mode in effect
int multi_set_gather(MultiDev* m, int64_t mode, std::string& err);
int64_t multi_gather(const MultiDev* m);
const char* multi_transport(const MultiDev* m);

// ---- render.hip ----
mrt_ctx* ctx_wrap_multi(MultiDev* m);  // the public handle of a multi-device context
MultiDev* ctx_multi(const mrt_ctx* c);  // null for a single-device context
void ctx_set_error(mrt_ctx* c, const std::string& msg);
void ctx_images(mrt_ctx* c, int delta);  // live mrt_image count of the handle (mrt_destroy refuses while > 0)
