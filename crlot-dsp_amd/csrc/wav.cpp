// wav.cpp -- WAV file I/O of the C ABI (include/crlot_dsp.h, "WAV I/O").
//
// Host-side replacement for the reference's io/wav.{h,cc} (WavReader /
// WavWriter over dr_wav, third_party/dr_libs -- an empty submodule, version
// unrecoverable).  Same guards as wav.cc:17-62 (1 or 2 channels; 16/24/32-bit
// PCM or 32-bit IEEE float), same float conversions as dr_wav's published
// drwav_read_pcm_frames_f32 / drwav_f32_to_s16 / drwav_f32_to_s32, and the
// reference's own 24-bit writer (wav.cc:233-246).  RIFF only (dr_wav also
// reads W64/RF64, which the reference never produces or tests).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "crlot_dsp.h"

namespace crlot {
int set_error(int code, const std::string& msg);  // abi.cpp: crlot_last_error()'s slot
}

namespace {

int wfail(int code, const std::string& msg) { return crlot::set_error(code, msg); }

uint16_t rd16(const unsigned char* p) { return uint16_t(p[0] | (p[1] << 8)); }
uint32_t rd32(const unsigned char* p) {
    return uint32_t(p[0]) | (uint32_t(p[1]) << 8) | (uint32_t(p[2]) << 16) | (uint32_t(p[3]) << 24);
}
void wr16(unsigned char* p, uint16_t v) {
    p[0] = uint8_t(v);
    p[1] = uint8_t(v >> 8);
}
void wr32(unsigned char* p, uint32_t v) {
    for (int i = 0; i < 4; ++i) p[i] = uint8_t(v >> (8 * i));
}

constexpr uint16_t kPcm = 1, kFloat = 3, kExtensible = 0xFFFE;

}  // namespace

struct crlot_wav_reader {
    FILE* f = nullptr;
    uint32_t channels = 0, sample_rate = 0, bits = 0;
    uint16_t format = 0;  // translated format tag: kPcm or kFloat
    uint64_t total_frames = 0, pos = 0;
    std::vector<unsigned char> scratch;
};

struct crlot_wav_writer {
    FILE* f = nullptr;
    uint32_t channels = 0, bits = 0;
    bool is_float = false;
    uint64_t data_bytes = 0;
    std::vector<unsigned char> scratch;
};

extern "C" {

int crlot_wav_reader_open(const char* path, crlot_wav_reader** out) {
    if (!path || !out) return wfail(CRLOT_EINVAL, "null argument");
    *out = nullptr;
    FILE* f = std::fopen(path, "rb");
    if (!f) return wfail(CRLOT_ERUNTIME, std::string("cannot open ") + path);
    auto bad = [&](const std::string& m) {
        std::fclose(f);
        return wfail(CRLOT_ERUNTIME, m);
    };
    unsigned char hdr[12];
    if (std::fread(hdr, 1, 12, f) != 12 || std::memcmp(hdr, "RIFF", 4) || std::memcmp(hdr + 8, "WAVE", 4))
        return bad("not a RIFF/WAVE file");
    bool have_fmt = false;
    uint16_t tag = 0, channels = 0, bits = 0, block_align = 0;
    uint32_t rate = 0;
    for (;;) {
        unsigned char ch[8];
        if (std::fread(ch, 1, 8, f) != 8) return bad("no data chunk");
        const uint32_t size = rd32(ch + 4);
        if (!std::memcmp(ch, "fmt ", 4)) {
            if (size < 16) return bad("fmt chunk too small");
            std::vector<unsigned char> fmt(size);
            if (std::fread(fmt.data(), 1, size, f) != size) return bad("truncated fmt chunk");
            tag = rd16(&fmt[0]);
            channels = rd16(&fmt[2]);
            rate = rd32(&fmt[4]);
            block_align = rd16(&fmt[12]);
            bits = rd16(&fmt[14]);
            if (tag == kExtensible && size >= 40) tag = rd16(&fmt[24]);  // SubFormat GUID's tag
            if (size & 1) std::fseek(f, 1, SEEK_CUR);
            have_fmt = true;
        } else if (!std::memcmp(ch, "data", 4)) {
            if (!have_fmt) return bad("data chunk before fmt chunk");
            // guards of WavReader::open (wav.cc:26-55)
            if (channels != 1 && channels != 2)
                return bad("unsupported channel count " + std::to_string(channels) +
                           " (mono=1 or stereo=2 only)");
            if (bits != 16 && bits != 24 && bits != 32)
                return bad("unsupported bit depth " + std::to_string(bits) + " (16, 24, 32 only)");
            if (!(tag == kPcm || (tag == kFloat && bits == 32)))
                return bad("unsupported format tag " + std::to_string(tag) + " (PCM or IEEE_FLOAT)");
            const uint32_t frame_bytes = uint32_t(channels) * (bits / 8);
            if (block_align != 0 && block_align != frame_bytes) return bad("unsupported block align");
            crlot_wav_reader* r = new crlot_wav_reader();
            r->f = f;
            r->channels = channels;
            r->sample_rate = rate;
            r->bits = bits;
            r->format = tag;
            r->total_frames = size / frame_bytes;
            *out = r;
            return CRLOT_OK;
        } else {
            if (std::fseek(f, long(size) + long(size & 1), SEEK_CUR)) return bad("truncated chunk");
        }
    }
}

void crlot_wav_reader_close(crlot_wav_reader* r) {
    if (!r) return;
    if (r->f) std::fclose(r->f);
    delete r;
}

int crlot_wav_reader_info(const crlot_wav_reader* r, uint32_t* channels, uint32_t* sample_rate,
                          uint64_t* total_frames, uint32_t* bits_per_sample, int32_t* is_float) {
    if (!r) return wfail(CRLOT_EINVAL, "null reader");
    if (channels) *channels = r->channels;
    if (sample_rate) *sample_rate = r->sample_rate;
    if (total_frames) *total_frames = r->total_frames;
    if (bits_per_sample) *bits_per_sample = r->bits;
    if (is_float) *is_float = r->format == kFloat;
    return CRLOT_OK;
}

// drwav_read_pcm_frames_f32: interleaved float frames from the current position.
int crlot_wav_reader_read(crlot_wav_reader* r, float* out, uint64_t frames, uint64_t* frames_read) {
    if (!r || (!out && frames)) return wfail(CRLOT_EINVAL, "null argument");
    const uint64_t left = r->total_frames - r->pos;
    const uint64_t n = frames < left ? frames : left;
    const size_t samples = size_t(n) * r->channels, bps = r->bits / 8;
    r->scratch.resize(samples * bps);
    const size_t got = samples ? std::fread(r->scratch.data(), bps, samples, r->f) : 0;
    const unsigned char* p = r->scratch.data();
    for (size_t i = 0; i < got; ++i, p += bps) {
        if (r->format == kFloat) {
            std::memcpy(&out[i], p, 4);
        } else if (bps == 2) {  // drwav_s16_to_f32: x * (1 / 32768)
            out[i] = float(int16_t(rd16(p))) * 0.000030517578125f;
        } else if (bps == 3) {  // drwav_s24_to_f32: sign-extended, scaled in double
            const int32_t v = int32_t((uint32_t(p[0]) << 8) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 24)) >> 8;
            out[i] = float(double(v) * 0.00000011920928955078125);
        } else {  // drwav_s32_to_f32: x / 2^31 in double
            out[i] = float(double(int32_t(rd32(p))) / 2147483648.0);
        }
    }
    const uint64_t done = got / r->channels;
    r->pos += done;
    if (frames_read) *frames_read = done;
    return CRLOT_OK;
}

int crlot_wav_writer_open(const char* path, uint32_t channels, uint32_t sample_rate,
                          uint32_t bits_per_sample, int32_t float_format, crlot_wav_writer** out) {
    if (!path || !out) return wfail(CRLOT_EINVAL, "null argument");
    *out = nullptr;
    // guards of WavWriter::open (wav.cc:170-180)
    if (channels != 1 && channels != 2)
        return wfail(CRLOT_ERUNTIME, "unsupported channel count " + std::to_string(channels));
    if (bits_per_sample != 16 && bits_per_sample != 24 && bits_per_sample != 32)
        return wfail(CRLOT_ERUNTIME, "unsupported bit depth " + std::to_string(bits_per_sample));
    FILE* f = std::fopen(path, "wb");
    if (!f) return wfail(CRLOT_ERUNTIME, std::string("cannot create ") + path);
    const bool is_float = float_format && bits_per_sample == 32;
    unsigned char h[44] = {};
    std::memcpy(h, "RIFF", 4);
    std::memcpy(h + 8, "WAVEfmt ", 8);
    wr32(h + 16, 16);
    wr16(h + 20, is_float ? kFloat : kPcm);
    wr16(h + 22, uint16_t(channels));
    wr32(h + 24, sample_rate);
    const uint32_t block = channels * (bits_per_sample / 8);
    wr32(h + 28, sample_rate * block);
    wr16(h + 32, uint16_t(block));
    wr16(h + 34, uint16_t(bits_per_sample));
    std::memcpy(h + 36, "data", 4);  // sizes patched on close
    if (std::fwrite(h, 1, 44, f) != 44) {
        std::fclose(f);
        return wfail(CRLOT_ERUNTIME, "write failed");
    }
    crlot_wav_writer* w = new crlot_wav_writer();
    w->f = f;
    w->channels = channels;
    w->bits = bits_per_sample;
    w->is_float = is_float;
    *out = w;
    return CRLOT_OK;
}

int crlot_wav_writer_write(crlot_wav_writer* w, const float* in, uint64_t frames, uint64_t* written) {
    if (!w || (!in && frames)) return wfail(CRLOT_EINVAL, "null argument");
    const size_t samples = size_t(frames) * w->channels, bps = w->bits / 8;
    w->scratch.resize(samples * bps);
    unsigned char* p = w->scratch.data();
    for (size_t i = 0; i < samples; ++i, p += bps) {
        const float x = in[i];
        if (w->is_float) {
            std::memcpy(p, &x, 4);
        } else if (bps == 2) {  // drwav_f32_to_s16
            const float c = (x < -1.0f ? -1.0f : (x > 1.0f ? 1.0f : x)) + 1.0f;
            wr16(p, uint16_t(int16_t(int(c * 32767.5f) - 32768)));
        } else if (bps == 3) {  // wav.cc:233-246
            const float c = std::fmax(-1.0f, std::fmin(1.0f, x));
            int32_t s = int32_t(std::lrintf(c * 8388607.0f));
            if (s > 8388607) s = 8388607;
            if (s < -8388608) s = -8388608;
            p[0] = uint8_t(s & 0xFF);
            p[1] = uint8_t((s >> 8) & 0xFF);
            p[2] = uint8_t((s >> 16) & 0xFF);
        } else {  // drwav_f32_to_s32: 2^31 * x (clamped here: 1.0 would overflow int32)
            const double d = 2147483648.0 * double(x);
            const int32_t s = d >= 2147483647.0 ? 2147483647 : d <= -2147483648.0 ? INT32_MIN : int32_t(d);
            wr32(p, uint32_t(s));
        }
    }
    const size_t put = samples ? std::fwrite(w->scratch.data(), 1, samples * bps, w->f) : 0;
    w->data_bytes += put;
    const uint64_t done = put / (bps * w->channels);
    if (written) *written = done;
    if (done != frames) return wfail(CRLOT_ERUNTIME, "short write");
    return CRLOT_OK;
}

int crlot_wav_writer_close(crlot_wav_writer* w) {
    if (!w) return CRLOT_OK;
    int rc = CRLOT_OK;
    if (w->f) {
        if (w->data_bytes & 1) std::fputc(0, w->f);  // RIFF chunks are word aligned
        unsigned char b[4];
        wr32(b, uint32_t(36 + w->data_bytes + (w->data_bytes & 1)));
        if (std::fseek(w->f, 4, SEEK_SET) || std::fwrite(b, 1, 4, w->f) != 4) rc = CRLOT_ERUNTIME;
        wr32(b, uint32_t(w->data_bytes));
        if (std::fseek(w->f, 40, SEEK_SET) || std::fwrite(b, 1, 4, w->f) != 4) rc = CRLOT_ERUNTIME;
        if (std::fclose(w->f)) rc = CRLOT_ERUNTIME;
    }
    delete w;
    return rc == CRLOT_OK ? rc : wfail(rc, "failed to finalise WAV header");
}

}  // extern "C"
