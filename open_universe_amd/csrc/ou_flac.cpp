// ou_flac.cpp -- FLAC stream decoder for the enhance CLI (host code).
//
// The reference CLI reads its inputs with torchaudio.load, which accepts
// .wav / .mp3 / .flac (open_universe/bin/enhance.py:33,61-64).  torchaudio and
// libFLAC are absent from this image, so FLAC (lossless, a fixed bitstream:
// RFC 9639) is decoded here into the planar float32 layout torchaudio.load
// returns: out[c][i] = sample / 2^(bps - 1).
//
// Covered: STREAMINFO, fixed and variable block sizes, every frame-header
// code (block size, sample rate, sample size, channel assignment), CONSTANT /
// VERBATIM / FIXED (order 0-4) / LPC (order 1-32) subframes, wasted bits,
// Rice partitions with 4- and 5-bit parameters and escape codes, the three
// stereo decorrelation modes, and both checksums (header CRC-8, frame
// CRC-16): a damaged stream fails loudly instead of decoding to noise.
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/ouhip.h"
#include "ou_common.h"

namespace {

struct Bits {
    const uint8_t* p;
    int64_t n;        // bytes
    int64_t pos = 0;  // bit position
    bool bad = false;

    uint32_t get(int k)   // k <= 32 bits, MSB first
    {
        uint64_t v = 0;
        for (int i = 0; i < k; ++i) {
            if (pos >= 8 * n) { bad = true; return 0; }
            v = (v << 1) | ((p[pos >> 3] >> (7 - (pos & 7))) & 1);
            ++pos;
        }
        return (uint32_t)v;
    }
    int32_t get_signed(int k)
    {
        if (k == 0) return 0;
        const uint32_t v = get(k);
        if (k == 32) return (int32_t)v;
        return (int32_t)(v << (32 - k)) >> (32 - k);
    }
    uint32_t unary()   // count of 0 bits before the next 1
    {
        uint32_t q = 0;
        while (!bad) {
            if (pos >= 8 * n) { bad = true; break; }
            if ((p[pos >> 3] >> (7 - (pos & 7))) & 1) { ++pos; break; }
            ++pos;
            ++q;
        }
        return q;
    }
    void align() { pos = (pos + 7) & ~(int64_t)7; }
};

uint8_t crc8(const uint8_t* d, int64_t n)
{
    uint8_t c = 0;
    for (int64_t i = 0; i < n; ++i) {
        c ^= d[i];
        for (int b = 0; b < 8; ++b) c = (uint8_t)((c & 0x80) ? (c << 1) ^ 0x07 : c << 1);
    }
    return c;
}

uint16_t crc16(const uint8_t* d, int64_t n)
{
    uint16_t c = 0;
    for (int64_t i = 0; i < n; ++i) {
        c ^= (uint16_t)d[i] << 8;
        for (int b = 0; b < 8; ++b) c = (uint16_t)((c & 0x8000) ? (c << 1) ^ 0x8005 : c << 1);
    }
    return c;
}

struct StreamInfo {
    int rate = 0, channels = 0, bps = 0;
    int64_t total = 0;
    int64_t first_frame = 0;   // byte offset of the first frame
};

int parse_header(const uint8_t* d, int64_t n, StreamInfo& si)
{
    if (n < 8 || std::memcmp(d, "fLaC", 4) != 0) return ou_fail(-1, "flac: missing fLaC marker");
    int64_t off = 4;
    bool have_info = false;
    for (;;) {
        if (off + 4 > n) return ou_fail(-1, "flac: truncated metadata");
        const bool last = d[off] & 0x80;
        const int type = d[off] & 0x7f;
        const int64_t len = ((int64_t)d[off + 1] << 16) | (d[off + 2] << 8) | d[off + 3];
        off += 4;
        if (off + len > n) return ou_fail(-1, "flac: truncated metadata block");
        if (type == 0) {
            if (len < 34) return ou_fail(-1, "flac: short STREAMINFO");
            Bits b{d + off, len};
            b.get(16);   // min block size
            b.get(16);   // max block size
            b.get(24);   // min frame size
            b.get(24);   // max frame size
            si.rate = (int)b.get(20);
            si.channels = (int)b.get(3) + 1;
            si.bps = (int)b.get(5) + 1;
            si.total = ((int64_t)b.get(4) << 32) | b.get(32);
            have_info = true;
        }
        off += len;
        if (last) break;
    }
    if (!have_info) return ou_fail(-1, "flac: no STREAMINFO block");
    si.first_frame = off;
    return 0;
}

// residual of one subframe into r[order ..] (r[0 .. order) holds the warm-up)
bool residual(Bits& b, int bsize, int order, int32_t* r)
{
    const int method = (int)b.get(2);
    if (method > 1) return false;
    const int pbits = method == 0 ? 4 : 5;
    const uint32_t escape = method == 0 ? 15u : 31u;
    const int porder = (int)b.get(4);
    const int parts = 1 << porder;
    if ((bsize >> porder) << porder != bsize || (bsize >> porder) < order) return false;
    int i = order;
    for (int pt = 0; pt < parts; ++pt) {
        const int cnt = (bsize >> porder) - (pt == 0 ? order : 0);
        const uint32_t k = b.get(pbits);
        if (k == escape) {
            const int raw = (int)b.get(5);
            for (int j = 0; j < cnt; ++j) r[i++] = b.get_signed(raw);
        } else {
            for (int j = 0; j < cnt; ++j) {
                const uint32_t q = b.unary();
                const uint32_t u = (q << k) | b.get((int)k);
                r[i++] = (int32_t)(u >> 1) ^ -(int32_t)(u & 1);
            }
        }
        if (b.bad) return false;
    }
    return true;
}

bool subframe(Bits& b, int bsize, int bps, int32_t* s)
{
    if (b.get(1) != 0) return false;
    const int type = (int)b.get(6);
    int wasted = 0;
    if (b.get(1)) wasted = (int)b.unary() + 1;
    const int eb = bps - wasted;
    if (eb <= 0 || eb > 32) return false;
    if (type == 0) {   // CONSTANT
        const int32_t v = b.get_signed(eb);
        for (int i = 0; i < bsize; ++i) s[i] = v;
    } else if (type == 1) {   // VERBATIM
        for (int i = 0; i < bsize; ++i) s[i] = b.get_signed(eb);
    } else if (type >= 8 && type <= 12) {   // FIXED, order 0..4
        const int order = type - 8;
        if (order > bsize) return false;
        for (int i = 0; i < order; ++i) s[i] = b.get_signed(eb);
        if (!residual(b, bsize, order, s)) return false;
        for (int i = order; i < bsize; ++i) {
            int64_t p = 0;
            switch (order) {
            case 1: p = s[i - 1]; break;
            case 2: p = 2 * (int64_t)s[i - 1] - s[i - 2]; break;
            case 3: p = 3 * (int64_t)s[i - 1] - 3 * (int64_t)s[i - 2] + s[i - 3]; break;
            case 4: p = 4 * (int64_t)s[i - 1] - 6 * (int64_t)s[i - 2] + 4 * (int64_t)s[i - 3] - s[i - 4]; break;
            }
            s[i] = (int32_t)(p + s[i]);
        }
    } else if (type >= 32) {   // LPC, order 1..32
        const int order = type - 31;
        if (order > bsize) return false;
        for (int i = 0; i < order; ++i) s[i] = b.get_signed(eb);
        const int prec = (int)b.get(4) + 1;
        if (prec == 16) return false;   // 0b1111 is invalid
        const int shift = b.get_signed(5);
        if (shift < 0) return false;
        int32_t c[32];
        for (int i = 0; i < order; ++i) c[i] = b.get_signed(prec);
        if (!residual(b, bsize, order, s)) return false;
        for (int i = order; i < bsize; ++i) {
            int64_t acc = 0;
            for (int j = 0; j < order; ++j) acc += (int64_t)c[j] * s[i - 1 - j];
            s[i] = (int32_t)((acc >> shift) + s[i]);
        }
    } else {
        return false;   // reserved subframe type
    }
    if (wasted)
        for (int i = 0; i < bsize; ++i) s[i] = (int32_t)((uint32_t)s[i] << wasted);
    return !b.bad;
}

const int kSizes[8] = {0, 8, 12, -1, 16, 20, 24, 32};

// Decodes every frame; out == nullptr counts frames only.
int64_t decode(const uint8_t* d, int64_t n, const StreamInfo& si, float* out, int64_t cap)
{
    int64_t off = si.first_frame, done = 0;
    std::vector<int32_t> ch[8];
    while (off + 2 <= n) {
        if (d[off] != 0xFF || (d[off + 1] & 0xFE) != 0xF8)
            return ou_fail(-2, "flac: lost frame sync at byte %lld", (long long)off);
        Bits b{d + off, n - off};
        b.get(16);
        const int bs_code = (int)b.get(4), sr_code = (int)b.get(4);
        const int ca = (int)b.get(4), ss_code = (int)b.get(3);
        b.get(1);
        // coded frame / sample number (UTF-8-like, 1..7 bytes)
        uint32_t lead = b.get(8);
        int extra = 0;
        while (extra < 7 && (lead & (0x80u >> extra))) ++extra;
        if (extra == 1 || extra > 7) return ou_fail(-2, "flac: bad coded number");
        for (int i = 1; i < extra; ++i) b.get(8);
        int bsize = 0;
        if (bs_code == 1) bsize = 192;
        else if (bs_code >= 2 && bs_code <= 5) bsize = 576 << (bs_code - 2);
        else if (bs_code == 6) bsize = (int)b.get(8) + 1;
        else if (bs_code == 7) bsize = (int)b.get(16) + 1;
        else if (bs_code >= 8) bsize = 256 << (bs_code - 8);
        else return ou_fail(-2, "flac: reserved block size code");
        if (sr_code == 12) b.get(8);
        else if (sr_code == 13 || sr_code == 14) b.get(16);
        else if (sr_code == 15) return ou_fail(-2, "flac: invalid sample rate code");
        const int bps = ss_code == 0 ? si.bps : kSizes[ss_code];
        if (bps <= 0) return ou_fail(-2, "flac: reserved sample size code");
        const int hdr_bytes = (int)(b.pos >> 3);
        if (b.bad || crc8(d + off, hdr_bytes) != b.get(8))
            return ou_fail(-2, "flac: frame header CRC-8 mismatch at byte %lld", (long long)off);
        const int nch = ca < 8 ? ca + 1 : 2;
        if (ca > 10) return ou_fail(-2, "flac: reserved channel assignment");
        if (nch != si.channels) return ou_fail(-2, "flac: frame has %d channels, stream %d", nch, si.channels);
        for (int c = 0; c < nch; ++c) {
            ch[c].resize(bsize);
            const bool side = (ca == 8 && c == 1) || (ca == 9 && c == 0) || (ca == 10 && c == 1);
            if (!subframe(b, bsize, bps + (side ? 1 : 0), ch[c].data()))
                return ou_fail(-2, "flac: bad subframe (channel %d) at byte %lld", c, (long long)off);
        }
        b.align();
        const int64_t body = b.pos >> 3;
        if (off + body + 2 > n) return ou_fail(-2, "flac: truncated frame");
        const uint16_t want = (uint16_t)((d[off + body] << 8) | d[off + body + 1]);
        if (crc16(d + off, body) != want)
            return ou_fail(-2, "flac: frame CRC-16 mismatch at byte %lld", (long long)off);
        off += body + 2;
        if (out) {
            if (done + bsize > cap) return ou_fail(-2, "flac: more samples than the output holds");
            const float scale = 1.0f / (float)(1u << (bps - 1));
            for (int i = 0; i < bsize; ++i) {
                int64_t v[8];
                for (int c = 0; c < nch; ++c) v[c] = ch[c][i];
                if (ca == 8) v[1] = v[0] - v[1];                 // left / side
                else if (ca == 9) v[0] = v[0] + v[1];            // side / right
                else if (ca == 10) {                             // mid / side
                    const int64_t mid = (v[0] * 2) | (v[1] & 1);
                    const int64_t sd = v[1];
                    v[0] = (mid + sd) >> 1;
                    v[1] = (mid - sd) >> 1;
                }
                for (int c = 0; c < nch; ++c) out[(int64_t)c * cap + done + i] = (float)v[c] * scale;
            }
        }
        done += bsize;
    }
    return done;
}

}  // namespace

extern "C" int ou_flac_info(const uint8_t* data, int64_t n, int32_t* sample_rate, int32_t* channels,
                            int32_t* bits_per_sample, int64_t* frames)
{
    if (!data || n <= 0) return ou_fail(-1, "flac: no data");
    StreamInfo si;
    const int rc = parse_header(data, n, si);
    if (rc) return rc;
    int64_t total = si.total;
    if (total == 0) {   // unknown in STREAMINFO: count the frames
        total = decode(data, n, si, nullptr, 0);
        if (total < 0) return (int)total;
    }
    if (sample_rate) *sample_rate = si.rate;
    if (channels) *channels = si.channels;
    if (bits_per_sample) *bits_per_sample = si.bps;
    if (frames) *frames = total;
    return 0;
}

extern "C" int64_t ou_flac_decode(const uint8_t* data, int64_t n, float* out, int64_t frames)
{
    if (!data || n <= 0 || !out || frames < 0) return ou_fail(-1, "flac: bad args");
    StreamInfo si;
    const int rc = parse_header(data, n, si);
    if (rc) return rc;
    return decode(data, n, si, out, frames);
}
