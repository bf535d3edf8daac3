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
#include <algorithm>
#include <cmath>
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
    int64_t get_signed64(int k)   // k <= 33 (a 32-bit stream's side channel)
    {
        if (k <= 32) return get_signed(k);
        const uint64_t hi = get(k - 32), lo = get(32);
        const uint64_t v = (hi << 32) | lo;
        return (int64_t)(v << (64 - k)) >> (64 - k);
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
bool residual(Bits& b, int bsize, int order, int64_t* r)
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
                r[i++] = (int64_t)((int32_t)(u >> 1) ^ -(int32_t)(u & 1));
            }
        }
        if (b.bad) return false;
    }
    return true;
}

// samples are int64: the side channel of a 32-bit stereo stream needs 33 bits
bool subframe(Bits& b, int bsize, int bps, int64_t* s)
{
    if (b.get(1) != 0) return false;
    const int type = (int)b.get(6);
    int wasted = 0;
    if (b.get(1)) wasted = (int)b.unary() + 1;
    const int eb = bps - wasted;
    if (eb <= 0 || eb > 33) return false;
    if (type == 0) {   // CONSTANT
        const int64_t v = b.get_signed64(eb);
        for (int i = 0; i < bsize; ++i) s[i] = v;
    } else if (type == 1) {   // VERBATIM
        for (int i = 0; i < bsize; ++i) s[i] = b.get_signed64(eb);
    } else if (type >= 8 && type <= 12) {   // FIXED, order 0..4
        const int order = type - 8;
        if (order > bsize) return false;
        for (int i = 0; i < order; ++i) s[i] = b.get_signed64(eb);
        if (!residual(b, bsize, order, s)) return false;
        for (int i = order; i < bsize; ++i) {
            int64_t p = 0;
            switch (order) {
            case 1: p = s[i - 1]; break;
            case 2: p = 2 * s[i - 1] - s[i - 2]; break;
            case 3: p = 3 * s[i - 1] - 3 * s[i - 2] + s[i - 3]; break;
            case 4: p = 4 * s[i - 1] - 6 * s[i - 2] + 4 * s[i - 3] - s[i - 4]; break;
            }
            s[i] = p + s[i];
        }
    } else if (type >= 32) {   // LPC, order 1..32
        const int order = type - 31;
        if (order > bsize) return false;
        for (int i = 0; i < order; ++i) s[i] = b.get_signed64(eb);
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
            s[i] = (acc >> shift) + s[i];
        }
    } else {
        return false;   // reserved subframe type
    }
    if (wasted)
        for (int i = 0; i < bsize; ++i) s[i] = (int64_t)((uint64_t)s[i] << wasted);
    return !b.bad;
}

const int kSizes[8] = {0, 8, 12, -1, 16, 20, 24, 32};

// Decodes every frame; out == nullptr counts frames only.
int64_t decode(const uint8_t* d, int64_t n, const StreamInfo& si, float* out, int64_t cap)
{
    int64_t off = si.first_frame, done = 0;
    std::vector<int64_t> ch[8];
    while (off + 2 <= n) {
        if (d[off] != 0xFF || (d[off + 1] & 0xFE) != 0xF8) {
            // bytes after the last frame (an ID3v1 'TAG' block, padding):
            // libFLAC / torchaudio.load stop there once every sample is in
            if ((si.total > 0 && done >= si.total) || (n - off >= 3 && std::memcmp(d + off, "TAG", 3) == 0))
                break;
            return ou_fail(-2, "flac: lost frame sync at byte %lld", (long long)off);
        }
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


// ---------------------------------------------------------------------------
// Encoder (the CLI writes a .flac output for a .flac input, as torchaudio.save
// does): PCM of bps bits (x * 2^(bps-1), rounded, clamped), blocks of 4096
// frames, independent channels, each subframe FIXED order 2 with one Rice
// partition, or VERBATIM when that is not smaller; STREAMINFO carries the
// total and a zero MD5 ("not computed", allowed by RFC 9639).
struct BitOut {
    std::vector<uint8_t> b;
    uint64_t acc = 0;
    int nacc = 0;
    void put(uint64_t v, int k)
    {
        for (int i = k - 1; i >= 0; --i) {
            acc = (acc << 1) | ((v >> i) & 1);
            if (++nacc == 8) { b.push_back((uint8_t)acc); acc = 0; nacc = 0; }
        }
    }
    void zeros(uint64_t q) { for (uint64_t i = 0; i < q; ++i) put(0, 1); }
    void align() { while (nacc) put(0, 1); }
};

constexpr int kEncBlock = 4096;

void put_utf8(BitOut& o, uint32_t n)
{
    if (n < 0x80) { o.put(n, 8); return; }
    int nb = 2;
    while (nb < 7 && n >= (1u << (5 * nb + 1))) ++nb;
    o.put(((0xFFu << (8 - nb)) & 0xFF) | (n >> (6 * (nb - 1))), 8);
    for (int i = nb - 2; i >= 0; --i) o.put(0x80 | ((n >> (6 * i)) & 0x3F), 8);
}

void enc_subframe(BitOut& o, const int32_t* s, int n, int bps)
{
    // FIXED order 2 residual and its Rice cost for the best parameter
    std::vector<uint32_t> u;
    uint64_t sum = 0;
    if (n > 2) {
        u.resize(n - 2);
        for (int i = 2; i < n; ++i) {
            const int64_t r = (int64_t)s[i] - (2 * (int64_t)s[i - 1] - s[i - 2]);
            const uint64_t z = r >= 0 ? (uint64_t)r << 1 : ((uint64_t)(-r) << 1) - 1;
            u[i - 2] = z > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)z;
            sum += u[i - 2];
        }
    }
    int k = 0;
    if (!u.empty()) {
        const uint64_t mean = sum / u.size();
        while (k < 30 && (1ull << (k + 1)) <= mean) ++k;
    }
    uint64_t bits = 2 * (uint64_t)bps + 2 + 4 + 5;
    for (uint32_t v : u) bits += (v >> k) + 1 + k;
    const bool fixed = n > 2 && bits < (uint64_t)n * bps;
    o.put(0, 1);
    o.put(fixed ? 8 + 2 : 1, 6);
    o.put(0, 1);   // no wasted bits
    if (!fixed) {
        for (int i = 0; i < n; ++i) o.put((uint32_t)s[i], bps);
        return;
    }
    o.put((uint32_t)s[0], bps);
    o.put((uint32_t)s[1], bps);
    o.put(1, 2);   // 5-bit Rice parameters
    o.put(0, 4);   // one partition
    o.put(k, 5);
    for (uint32_t v : u) {
        o.zeros(v >> k);
        o.put(1, 1);
        o.put(v, k);
    }
}

}  // namespace

extern "C" int64_t ou_flac_encode_bound(int channels, int64_t frames, int bps)
{
    const int64_t blocks = (frames + kEncBlock - 1) / kEncBlock;
    return 42 + blocks * (20 + (int64_t)channels * 8) + (int64_t)channels * frames * ((bps + 7) / 8);
}

extern "C" int64_t ou_flac_encode(const float* x, int channels, int64_t frames, int sample_rate, int bps,
                                  uint8_t* out, int64_t capacity)
{
    if (!x || !out || channels < 1 || channels > 8 || frames < 1 || (bps != 16 && bps != 24) ||
        sample_rate < 1 || sample_rate >= (1 << 20))
        return ou_fail(-1, "flac encode: bad args");
    BitOut o;
    o.b.reserve((size_t)std::min<int64_t>(capacity, ou_flac_encode_bound(channels, frames, bps)));
    for (const char* m = "fLaC"; *m; ++m) o.put((uint8_t)*m, 8);
    o.put(0x80, 8);   // last metadata block, STREAMINFO
    o.put(34, 24);
    const int first = (int)std::min<int64_t>(frames, kEncBlock);
    o.put(frames <= kEncBlock ? first : kEncBlock, 16);
    o.put(first, 16);
    o.put(0, 24);
    o.put(0, 24);
    o.put(sample_rate, 20);
    o.put(channels - 1, 3);
    o.put(bps - 1, 5);
    o.put((uint64_t)frames, 36);
    for (int i = 0; i < 16; ++i) o.put(0, 8);
    const double full = (double)(1 << (bps - 1));
    const int32_t lo = -(1 << (bps - 1)), hi = (1 << (bps - 1)) - 1;
    std::vector<int32_t> s(kEncBlock);
    uint32_t fno = 0;
    for (int64_t t0 = 0; t0 < frames; t0 += kEncBlock, ++fno) {
        const int n = (int)std::min<int64_t>(kEncBlock, frames - t0);
        const size_t start = o.b.size();
        o.put(0x3FFE, 14);
        o.put(0, 2);
        o.put(n == kEncBlock ? 12 : 7, 4);   // 4096 from the table, else 16-bit n - 1
        o.put(0, 4);                         // sample rate from STREAMINFO
        o.put(channels - 1, 4);
        o.put(bps == 16 ? 4 : 6, 3);
        o.put(0, 1);
        put_utf8(o, fno);
        if (n != kEncBlock) o.put(n - 1, 16);
        o.put(crc8(o.b.data() + start, (int64_t)(o.b.size() - start)), 8);
        for (int c = 0; c < channels; ++c) {
            for (int i = 0; i < n; ++i) {
                const double v = std::nearbyint((double)x[(int64_t)c * frames + t0 + i] * full);
                s[i] = (int32_t)std::max<double>(lo, std::min<double>(hi, v));
            }
            enc_subframe(o, s.data(), n, bps);
        }
        o.align();
        const uint16_t crc = crc16(o.b.data() + start, (int64_t)(o.b.size() - start));
        o.put(crc, 16);
    }
    if ((int64_t)o.b.size() > capacity) return ou_fail(-2, "flac encode: output needs %lld bytes", (long long)o.b.size());
    std::memcpy(out, o.b.data(), o.b.size());
    return (int64_t)o.b.size();
}

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
