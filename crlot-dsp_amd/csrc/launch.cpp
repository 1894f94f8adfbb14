// launch.cpp -- per-call launch knobs and launch records (kernels.h LaunchCtl),
// and the names of the CRLOT_K_* kernel ids (include/crlot_dsp.h).
#include <algorithm>
#include <cstdint>

#include "crlot_dsp.h"
#include "kernels.h"

namespace crlot {
namespace {
thread_local LaunchCtl* tl_ctl = nullptr;
}

LaunchCtl* launch_ctl() { return tl_ctl; }
void set_launch_ctl(LaunchCtl* c) { tl_ctl = c; }

void note_launch(int32_t id, int64_t grid) {
    LaunchCtl* c = tl_ctl;
    if (!c) return;
    LaunchRecord& r = c->rec;
    if (r.n < kLaunchRecordMax) {
        r.id[r.n] = id;
        r.grid[r.n] = grid;
    }
    ++r.n;
}

void note_chunks(int64_t n_chunks) {
    if (tl_ctl) tl_ctl->rec.n_chunks = int32_t(n_chunks);
}

int64_t chunks_or(int64_t dflt, int64_t max_chunks) {
    const LaunchCtl* c = tl_ctl;
    if (!c || c->chunks <= 0) return dflt;
    return std::max<int64_t>(1, std::min<int64_t>(c->chunks, max_chunks));
}

}  // namespace crlot

extern "C" const char* crlot_kernel_name(int32_t id) {
    switch (id) {
        case CRLOT_K_PAIR_HOT: return "k_pair_hot";
        case CRLOT_K_PAIR_FIX: return "k_pair_fix";
        case CRLOT_K_PAIR_ALL: return "k_pair_all";
        case CRLOT_K_PAIR512_HOT: return "k_pair512_hot";
        case CRLOT_K_PAIR512: return "k_pair512";
        case CRLOT_K_PAIR2K_HOT: return "k_pair2k_hot";
        case CRLOT_K_PAIR2K: return "k_pair2k";
        case CRLOT_K_PAIR4K_HOT: return "k_pair4k_hot";
        case CRLOT_K_PAIR4K: return "k_pair4k";
        case CRLOT_K_FUSED: return "k_fused";
        case CRLOT_K_FUSED2: return "k_fused2";
        case CRLOT_K_FUSED_WG: return "k_fused_wg";
        case CRLOT_K_PAIR15: return "k_pair15";
        case CRLOT_K_PAIRN: return "k_pairn";
        case CRLOT_K_PAIR30: return "k_pair30";
        case CRLOT_K_FUSED_ANY: return "k_fused_any";
        case CRLOT_K_SYNTH: return "k_synth";
        case CRLOT_K_SYNTH_ANY: return "k_synth_any";
        case CRLOT_K_GATHER: return "k_gather";
        case CRLOT_K_DEINTERLEAVE: return "k_deinterleave";
        case CRLOT_K_INTERLEAVE: return "k_interleave";
        case CRLOT_K_FFT: return "k_fft";
        case CRLOT_K_FFT_ANY: return "k_fft_any";
        case CRLOT_K_STFT: return "k_stft";
        case CRLOT_K_ISTFT: return "k_istft";
        case CRLOT_K_STFT_MASKED: return "k_stft_masked";
        case CRLOT_K_SPEC_STEP: return "k_spec_step";
        case CRLOT_K_FRAMES_W: return "k_frames_w";
        case CRLOT_K_PAIR_MASK: return "k_pair_mask";
        case CRLOT_K_PAIR_STFT: return "k_pair_stft";
        case CRLOT_K_PAIR_ISTFT: return "k_pair_istft";
        case CRLOT_K_EXPERIMENT: return "k_experiment";
        default: return "unknown";
    }
}
