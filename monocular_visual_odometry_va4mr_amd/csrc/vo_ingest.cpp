// Host-side frame ingest for the VO hot path: decode the dataset PNGs
// the reference reads with cv2.imread(path, cv2.IMREAD_GRAYSCALE) (utils.py:55-81) on a
// pool of host threads, straight into caller-provided (pinned) memory, so that decoding the
// next batch overlaps the GPU step of the current one.
//
// PNG: 8-bit gray / gray+alpha / RGB / RGBA / palette, non-interlaced, all five row filters.
// Colour images become gray the way OpenCV's PNG decoder asks libpng to do it
// (png_set_rgb_to_gray(1, 0.299, 0.587)), restated from libpng 1.6's integer path without
// gamma: the weights are fixed to 1e-5 units (29900, 58700) and scaled to 15 bits by
// truncation, (w * 32768) / 100000 -> red 9797, green 19234, blue 32768 - red - green = 3737;
// a pixel is (rc*R + gc*G + bc*B) >> 15 (truncating), and a pixel with R == G == B is passed
// through unchanged.  Parity with libpng / OpenCV unpinned (neither is in this image).
// 16-bit images keep the high byte (png_set_strip_16).
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <zlib.h>

#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace {

enum { ING_OK = 0, ING_EARG = -1, ING_EIO = -3, ING_EFORMAT = -4, ING_ESIZE = -5, ING_EZLIB = -6 };

uint32_t be32(const uint8_t* p) { return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]; }

struct PngHdr {
    uint32_t w = 0, h = 0;
    int depth = 0, ctype = 0, interlace = 0;
    int channels = 0;
};

int parse_header(const uint8_t* d, size_t n, PngHdr& h)
{
    static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    if (n < 33 || memcmp(d, sig, 8) != 0) return ING_EFORMAT;
    if (be32(d + 8) != 13 || memcmp(d + 12, "IHDR", 4) != 0) return ING_EFORMAT;
    h.w = be32(d + 16);
    h.h = be32(d + 20);
    h.depth = d[24];
    h.ctype = d[25];
    h.interlace = d[28];
    switch (h.ctype) {
        case 0: h.channels = 1; break;
        case 2: h.channels = 3; break;
        case 3: h.channels = 1; break;
        case 4: h.channels = 2; break;
        case 6: h.channels = 4; break;
        default: return ING_EFORMAT;
    }
    if (h.interlace != 0) return ING_EFORMAT;
    if (!(h.depth == 8 || (h.depth == 16 && h.ctype != 3))) return ING_EFORMAT;
    if (h.w == 0 || h.h == 0 || h.w > 65535 || h.h > 65535) return ING_EFORMAT;
    return ING_OK;
}

int paeth(int a, int b, int c)
{
    const int p = a + b - c;
    const int pa = p > a ? p - a : a - p, pb = p > b ? p - b : b - p, pc = p > c ? p - c : c - p;
    if (pa <= pb && pa <= pc) return a;
    return pb <= pc ? b : c;
}

constexpr int GRAY_RC = (29900 * 32768) / 100000;             // 9797
constexpr int GRAY_GC = (58700 * 32768) / 100000;             // 19234
constexpr int GRAY_BC = 32768 - GRAY_RC - GRAY_GC;            // 3737
inline uint8_t rgb_to_gray(int r, int g, int b)
{
    if (r == g && r == b) return (uint8_t)r;
    return (uint8_t)((GRAY_RC * r + GRAY_GC * g + GRAY_BC * b) >> 15);
}

int decode_png(const uint8_t* d, size_t n, uint8_t* out, int64_t pitch, int want_w, int want_h)
{
    PngHdr h;
    int rc = parse_header(d, n, h);
    if (rc) return rc;
    if ((int)h.w != want_w || (int)h.h != want_h) return ING_ESIZE;
    // concatenate IDAT, read PLTE
    std::vector<uint8_t> idat;
    uint8_t pal[256][3];
    int npal = 0;
    size_t p = 8;
    while (p + 12 <= n) {
        const uint32_t len = be32(d + p);
        const uint8_t* type = d + p + 4;
        if (p + 12 + (size_t)len > n) return ING_EFORMAT;
        const uint8_t* body = d + p + 8;
        if (!memcmp(type, "IDAT", 4)) idat.insert(idat.end(), body, body + len);
        else if (!memcmp(type, "PLTE", 4)) {
            npal = (int)(len / 3);
            if (npal > 256) npal = 256;
            for (int i = 0; i < npal; ++i) { pal[i][0] = body[3 * i]; pal[i][1] = body[3 * i + 1]; pal[i][2] = body[3 * i + 2]; }
        } else if (!memcmp(type, "IEND", 4)) break;
        p += 12 + (size_t)len;
    }
    const int bpp = h.channels * (h.depth / 8);           // bytes per pixel
    const size_t stride = (size_t)h.w * bpp;
    std::vector<uint8_t> raw((stride + 1) * h.h);
    z_stream zs;
    memset(&zs, 0, sizeof zs);
    if (inflateInit(&zs) != Z_OK) return ING_EZLIB;
    zs.next_in = idat.data();
    zs.avail_in = (uInt)idat.size();
    zs.next_out = raw.data();
    zs.avail_out = (uInt)raw.size();
    const int zr = inflate(&zs, Z_FINISH);
    inflateEnd(&zs);
    if (zr != Z_STREAM_END || zs.avail_out != 0) return ING_EZLIB;
    // unfilter row by row (filter type hoisted out of the byte loop); 8-bit gray rows are
    // reconstructed in place in the output
    const bool direct = (h.ctype == 0 && h.depth == 8);
    std::vector<uint8_t> zero(stride, 0), bufA(direct ? 0 : stride), bufB(direct ? 0 : stride);
    const uint8_t* prev = zero.data();
    for (uint32_t y = 0; y < h.h; ++y) {
        const uint8_t* row = raw.data() + y * (stride + 1);
        const int f = row[0];
        const uint8_t* src = row + 1;
        uint8_t* cur = direct ? out + (int64_t)y * pitch : ((y & 1) ? bufB.data() : bufA.data());
        const size_t B = (size_t)bpp;
        switch (f) {
            case 0:
                memcpy(cur, src, stride);
                break;
            case 1:
                for (size_t i = 0; i < B; ++i) cur[i] = src[i];
                for (size_t i = B; i < stride; ++i) cur[i] = (uint8_t)(src[i] + cur[i - B]);
                break;
            case 2:
                for (size_t i = 0; i < stride; ++i) cur[i] = (uint8_t)(src[i] + prev[i]);
                break;
            case 3:
                for (size_t i = 0; i < B; ++i) cur[i] = (uint8_t)(src[i] + (prev[i] >> 1));
                for (size_t i = B; i < stride; ++i) cur[i] = (uint8_t)(src[i] + ((cur[i - B] + prev[i]) >> 1));
                break;
            case 4:
                for (size_t i = 0; i < B; ++i) cur[i] = (uint8_t)(src[i] + prev[i]);
                for (size_t i = B; i < stride; ++i) cur[i] = (uint8_t)(src[i] + paeth(cur[i - B], prev[i], prev[i - B]));
                break;
            default:
                return ING_EFORMAT;
        }
        if (!direct) {
            uint8_t* o = out + (int64_t)y * pitch;
            const int s = h.depth / 8;                       // 16-bit: high byte first
            for (uint32_t x = 0; x < h.w; ++x) {
                const uint8_t* px = cur + (size_t)x * bpp;
                switch (h.ctype) {
                    case 0: case 4: o[x] = px[0]; break;
                    case 2: case 6: o[x] = rgb_to_gray(px[0], px[s], px[2 * s]); break;
                    case 3: {
                        const int k = px[0] < npal ? px[0] : 0;
                        o[x] = rgb_to_gray(pal[k][0], pal[k][1], pal[k][2]);
                        break;
                    }
                }
            }
        }
        prev = cur;
    }
    return ING_OK;
}

int read_file(const char* path, std::vector<uint8_t>& buf)
{
    FILE* f = fopen(path, "rb");
    if (!f) return ING_EIO;
    if (fseek(f, 0, SEEK_END) != 0) { fclose(f); return ING_EIO; }
    const long n = ftell(f);
    if (n <= 0) { fclose(f); return ING_EIO; }
    rewind(f);
    buf.resize((size_t)n);
    const size_t got = fread(buf.data(), 1, (size_t)n, f);
    fclose(f);
    return got == (size_t)n ? ING_OK : ING_EIO;
}

// fixed pool of worker threads that run indexed jobs
class Pool {
public:
    explicit Pool(int n)
    {
        for (int i = 0; i < n; ++i) th_.emplace_back([this] { loop(); });
    }
    ~Pool()
    {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    // run fn(i) for i in [0, n) on the pool; blocks until done
    void run(int n, const std::function<void(int)>& fn)
    {
        std::unique_lock<std::mutex> g(m_);
        fn_ = &fn;
        next_ = 0;
        total_ = n;
        done_ = 0;
        ++gen_;
        cv_.notify_all();
        done_cv_.wait(g, [&] { return done_ == total_; });
        fn_ = nullptr;
    }

private:
    void loop()
    {
        uint64_t seen = 0;
        std::unique_lock<std::mutex> g(m_);
        for (;;) {
            cv_.wait(g, [&] { return stop_ || (gen_ != seen && next_ < total_); });
            if (stop_) return;
            seen = gen_;
            while (next_ < total_) {
                const int i = next_++;
                const std::function<void(int)>* fn = fn_;
                g.unlock();
                (*fn)(i);
                g.lock();
                if (++done_ == total_) done_cv_.notify_all();
            }
        }
    }
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_cv_;
    const std::function<void(int)>* fn_ = nullptr;
    int next_ = 0, total_ = 0, done_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

}  // namespace

extern "C" {

// PNG header: width, height, channels (after palette expansion: 1 for palette), bit depth
int vo_png_info(const uint8_t* data, size_t len, int* w, int* h, int* channels, int* depth)
{
    if (!data) return ING_EARG;
    PngHdr hd;
    const int rc = parse_header(data, len, hd);
    if (rc) return rc;
    if (w) *w = (int)hd.w;
    if (h) *h = (int)hd.h;
    if (channels) *channels = hd.channels;
    if (depth) *depth = hd.depth;
    return ING_OK;
}

// cv2.imread(IMREAD_GRAYSCALE) of an in-memory PNG into out[h][pitch]
int vo_png_decode_gray(const uint8_t* data, size_t len, uint8_t* out, int64_t pitch, int w, int h)
{
    if (!data || !out || pitch < w) return ING_EARG;
    return decode_png(data, len, out, pitch, w, h);
}

void* vo_ingest_create(int n_threads)
{
    if (n_threads < 1) n_threads = 1;
    return new Pool(n_threads);
}

void vo_ingest_destroy(void* pool) { delete (Pool*)pool; }

// Decode n PNG files into out + i*frame_stride (each W x H, pitch W) on the pool; status[i]
// receives each file's code.  Returns 0 if every file decoded.  Blocks the caller (ctypes
// releases the GIL, so a Python thread can run this while the GPU steps).
int vo_ingest_png_files(void* pool, const char* const* paths, int n, uint8_t* out, int64_t frame_stride,
                        int W, int H, int32_t* status)
{
    if (!pool || !paths || !out || n < 0 || W < 1 || H < 1) return ING_EARG;
    std::atomic<int> bad{0};
    ((Pool*)pool)->run(n, [&](int i) {
        std::vector<uint8_t> buf;
        int rc = read_file(paths[i], buf);
        if (!rc) rc = decode_png(buf.data(), buf.size(), out + (int64_t)i * frame_stride, W, W, H);
        if (status) status[i] = rc;
        if (rc) bad.fetch_add(1);
    });
    return bad.load() ? ING_EFORMAT : ING_OK;
}

}  // extern "C"
