// tmpt_host.cpp -- host side of the drop-in: scene ingest, camera placement and
// the PNG writer.  Not kernels; these keep the reference's behaviour so the
// device path sees exactly the triangles and camera the reference would.
//
//  * load_obj       LoadScene (main.cpp:122-170) over objParseFile
//                   (objparser.cpp:304-355): 'v' and 'f' records, fan
//                   triangulation, negative indices, the floating-point
//                   parse of objparser.cpp:62-131 (digits accumulated in
//                   double, scaled by an exact power-of-ten table), then the
//                   two floor triangles 0.7x beyond the bounds.
//  * camera         Camera::Camera (maths.cpp:40-59) and the placement of
//                   main.cpp:295-307, in the GLM rounding order (tmpt_math.h).
//  * write_png      stbi_write_png with flip-on-write (main.cpp:341-342); the
//                   encoder is zlib's, so the file bytes differ from stb's but
//                   the decoded pixels are the same.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <string>
#include <thread>
#include <vector>

#include "tmpt.h"
#include "tmpt_math.h"

namespace tmpt {

void set_error(const std::string& msg);

namespace {

struct Cursor {
    const char* p;
    const char* end;
};

inline bool is_digit(char c) { return (unsigned)(c - '0') < 10u; }
inline void skip_blank(Cursor& c)
{
    while (c.p < c.end && (*c.p == ' ' || *c.p == '\t')) ++c.p;
}
inline char at(const Cursor& c) { return c.p < c.end ? *c.p : '\0'; }

// decimal integer with optional sign (objparser.cpp:34-60 semantics)
int read_int(Cursor& c)
{
    skip_blank(c);
    bool neg = at(c) == '-';
    if (at(c) == '-' || at(c) == '+') ++c.p;
    unsigned v = 0;
    while (is_digit(at(c))) v = v * 10u + (unsigned)(*c.p++ - '0');
    return neg ? -(int)v : (int)v;
}

// objparser.cpp:62-131 semantics: mantissa digits in double, decimal exponent
// applied through an exact 1e0..1e22 table, rounded once to float.
float read_float(Cursor& c)
{
    static const double kPow10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,
                                      1e8,  1e9,  1e10, 1e11, 1e12, 1e13, 1e14, 1e15,
                                      1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
    skip_blank(c);
    double sign = at(c) == '-' ? -1.0 : 1.0;
    if (at(c) == '-' || at(c) == '+') ++c.p;
    double m = 0.0;
    int e10 = 0;
    while (is_digit(at(c))) m = m * 10.0 + (double)(*c.p++ - '0');
    if (at(c) == '.') {
        ++c.p;
        while (is_digit(at(c))) {
            m = m * 10.0 + (double)(*c.p++ - '0');
            --e10;
        }
    }
    if ((at(c) | ' ') == 'e') {
        ++c.p;
        int es = at(c) == '-' ? -1 : 1;
        if (at(c) == '-' || at(c) == '+') ++c.p;
        int ev = 0;
        while (is_digit(at(c))) ev = ev * 10 + (*c.p++ - '0');
        e10 += es * ev;
    }
    if ((unsigned)(-e10) < 23u) return (float)(sign * m / kPow10[-e10]);
    if ((unsigned)e10 < 23u) return (float)(sign * m * kPow10[e10]);
    return (float)(sign * m * std::pow(10.0, e10));
}

// one "v[/vt][/vn]" group; only the position index is used downstream
int read_face_vertex(Cursor& c)
{
    skip_blank(c);
    int vi = read_int(c);
    if (at(c) == '/') {
        ++c.p;
        if (at(c) != '/') (void)read_int(c);
        if (at(c) == '/') {
            ++c.p;
            (void)read_int(c);
        }
    }
    return vi;
}

// Environment knobs of the parallel host paths (tests force small chunks).
int env_int(const char* name, int dflt)
{
    const char* e = getenv(name);
    return e && *e ? atoi(e) : dflt;
}

int host_threads(const char* env)
{
    int t = env_int(env, 0);
    if (t > 0) return t;
    unsigned hw = std::thread::hardware_concurrency();
    return (int)std::max(1u, std::min(16u, hw));
}

// One text chunk of an OBJ file parsed on its own: positions, and faces whose
// negative (relative) indices are resolved against the chunk-local vertex
// count and fixed up once the vertex counts of the earlier chunks are known.
struct ObjChunk {
    std::vector<float> pos;
    std::vector<int32_t> faces;
    std::vector<uint32_t> rel;  // indices into faces holding chunk-relative values
};

void parse_obj_chunk(const char* p, const char* end, ObjChunk& out)
{
    while (p < end) {
        const char* eol = (const char*)memchr(p, '\n', (size_t)(end - p));
        const char* le = eol ? eol : end;
        Cursor c{p, le};
        if (le - p >= 2 && p[0] == 'v' && p[1] == ' ') {
            c.p += 2;
            float x = read_float(c), y = read_float(c), z = read_float(c);
            out.pos.push_back(x);
            out.pos.push_back(y);
            out.pos.push_back(z);
        } else if (le - p >= 2 && p[0] == 'f' && p[1] == ' ') {
            c.p += 2;
            const int nv = (int)(out.pos.size() / 3);
            int fan0 = 0, prev = 0, k = 0;
            bool rfan0 = false, rprev = false;
            while (c.p < c.end) {
                int vi = read_face_vertex(c);
                if (vi == 0) break;
                const bool r = vi < 0;
                int idx = r ? nv + vi : vi - 1;  // objparser.cpp:29-32 (rel: + chunk base)
                if (k == 0) {
                    fan0 = idx;
                    rfan0 = r;
                } else if (k >= 2) {
                    const int v3[3] = {fan0, prev, idx};
                    const bool r3[3] = {rfan0, rprev, r};
                    for (int j = 0; j < 3; ++j) {
                        if (r3[j]) out.rel.push_back((uint32_t)out.faces.size());
                        out.faces.push_back(v3[j]);
                    }
                }
                prev = idx;
                rprev = r;
                ++k;
            }
        }
        p = le + 1;
    }
}

}  // namespace

// objParseFile (objparser.cpp:304-355) + the triangle gather of LoadScene,
// parallel: the text is cut at line starts into chunks parsed concurrently;
// chunk results are concatenated in file order, so the triangles are exactly
// those of a sequential parse ("parallel OBJ ingest").
int load_obj(const char* path, std::vector<float>& tris, f3& bmin, f3& bmax)
{
    FILE* f = fopen(path, "rb");
    if (!f) {
        set_error(std::string("cannot open '") + (path ? path : "") + "'");
        return -1;
    }
    std::string text;
    if (fseek(f, 0, SEEK_END) == 0) {
        long sz = ftell(f);
        if (sz > 0) text.resize((size_t)sz);
        fseek(f, 0, SEEK_SET);
    }
    size_t got = text.empty() ? 0 : fread(&text[0], 1, text.size(), f);
    text.resize(got);
    {  // files whose size ftell cannot tell (pipes): read to the end
        char buf[1 << 16];
        size_t more;
        while ((more = fread(buf, 1, sizeof(buf), f)) > 0) text.append(buf, more);
    }
    fclose(f);

    const char* base = text.data();
    const size_t len = text.size();
    const size_t min_chunk = (size_t)std::max(1, env_int("TMPT_OBJ_CHUNK", 1 << 20));
    const int nthreads = host_threads("TMPT_OBJ_THREADS");
    size_t nchunks = std::max<size_t>(1, std::min<size_t>((size_t)nthreads * 4, len / min_chunk));
    std::vector<size_t> cut(nchunks + 1, len);
    cut[0] = 0;
    for (size_t k = 1; k < nchunks; ++k) {  // chunk k starts at the line after byte k*len/n
        size_t at = std::max(cut[k - 1], k * len / nchunks);
        const char* nl = at < len ? (const char*)memchr(base + at, '\n', len - at) : nullptr;
        cut[k] = nl ? (size_t)(nl - base) + 1 : len;
    }
    std::vector<ObjChunk> chunks(nchunks);
    {
        std::atomic<size_t> next{0};
        auto work = [&]() {
            for (size_t k; (k = next.fetch_add(1)) < nchunks;)
                parse_obj_chunk(base + cut[k], base + cut[k + 1], chunks[k]);
        };
        std::vector<std::thread> pool;
        const int nt = (int)std::min<size_t>((size_t)nthreads, nchunks);
        for (int t = 1; t < nt; ++t) pool.emplace_back(work);
        work();
        for (auto& t : pool) t.join();
    }
    std::vector<float> pos;
    std::vector<int32_t> faces;
    {
        size_t np = 0, nf = 0;
        for (auto& ch : chunks) {
            np += ch.pos.size();
            nf += ch.faces.size();
        }
        pos.reserve(np);
        faces.reserve(nf);
        int32_t vbase = 0;
        for (auto& ch : chunks) {
            const size_t f0 = faces.size();
            pos.insert(pos.end(), ch.pos.begin(), ch.pos.end());
            faces.insert(faces.end(), ch.faces.begin(), ch.faces.end());
            for (uint32_t r : ch.rel) faces[f0 + r] += vbase;
            vbase += (int32_t)(ch.pos.size() / 3);
            std::vector<float>().swap(ch.pos);
            std::vector<int32_t>().swap(ch.faces);
        }
    }
    // LoadScene, main.cpp:132-162
    const size_t n = faces.size() / 3;
    const size_t nverts = pos.size() / 3;
    for (size_t i = 0; i < faces.size(); ++i) {
        if (faces[i] < 0 || (size_t)faces[i] >= nverts) {
            set_error("face index out of range in '" + std::string(path) + "'");
            return -2;
        }
    }
    bmin = mk(+1.0e6f, +1.0e6f, +1.0e6f);
    bmax = mk(-1.0e6f, -1.0e6f, -1.0e6f);
    tris.resize((n + 2) * 9);
    for (size_t i = 0; i < n; ++i) {
        for (int k = 0; k < 3; ++k) {
            const float* v = &pos[3 * (size_t)faces[3 * i + k]];
            tris[9 * i + 3 * k + 0] = v[0];
            tris[9 * i + 3 * k + 1] = v[1];
            tris[9 * i + 3 * k + 2] = v[2];
        }
        for (int k = 0; k < 3; ++k) {
            f3 v = mk(tris[9 * i + 3 * k], tris[9 * i + 3 * k + 1], tris[9 * i + 3 * k + 2]);
            bmin = vmin(bmin, v);
            bmax = vmax(bmax, v);
        }
    }
    f3 size = bmax - bmin;
    f3 extra = size * 0.7f;
    const float x0 = bmin.x - extra.x, x1 = bmax.x + extra.x;
    const float z0 = bmin.z - extra.z, z1 = bmax.z + extra.z, y = bmin.y;
    const float floor_tris[18] = {x0, y, z0, x0, y, z1, x1, y, z0,   // main.cpp:157-159
                                  x0, y, z1, x1, y, z1, x1, y, z0};  // main.cpp:160-162
    memcpy(&tris[9 * n], floor_tris, sizeof(floor_tris));
    return 0;
}

void camera_init(tmpt_camera* cam, f3 lookFrom, f3 lookAt, f3 vup, float vfov, float aspect,
                 float aperture, float focusDist)
{
    // Camera::Camera, maths.cpp:40-59
    cam->lens_radius = aperture * 0.5f;
    float theta = vfov * kPI / 180.0f;
    float halfHeight = tanf(theta * 0.5f);
    float halfWidth = aspect * halfHeight;
    f3 origin = lookFrom;
    f3 w = normalize(lookFrom - lookAt);
    f3 u = normalize(cross(vup, w));
    f3 v = cross(w, u);
    f3 llc = origin - halfWidth * focusDist * u - halfHeight * focusDist * v - focusDist * w;
    f3 hor = 2.0f * halfWidth * focusDist * u;
    f3 ver = 2.0f * halfHeight * focusDist * v;
    auto put = [](float* d, f3 s) { d[0] = s.x; d[1] = s.y; d[2] = s.z; };
    put(cam->origin, origin);
    put(cam->lower_left, llc);
    put(cam->horizontal, hor);
    put(cam->vertical, ver);
    put(cam->u, u);
    put(cam->v, v);
    put(cam->w, w);
}

void camera_for_scene(tmpt_camera* cam, f3 sceneMin, f3 sceneMax, int w, int h, bool sponza)
{
    // main.cpp:295-307
    f3 sceneSize = sceneMax - sceneMin;
    f3 sceneCenter = (sceneMin + sceneMax) * 0.5f;
    f3 lookfrom = sceneCenter + sceneSize * mk(0.3f, 0.6f, 1.2f);
    if (sponza) lookfrom = mk(-5.96f, 4.08f, -1.22f);
    f3 lookat = sceneCenter + sceneSize * mk(0.0f, -0.1f, 0.0f);
    const float distToFocus = length(lookfrom - lookat);
    camera_init(cam, lookfrom, lookat, mk(0.0f, 1.0f, 0.0f), 60.0f, float(w) / float(h), 0.03f,
                distToFocus);
}

namespace {
void be32(std::vector<uint8_t>& o, uint32_t v)
{
    o.push_back((uint8_t)(v >> 24));
    o.push_back((uint8_t)(v >> 16));
    o.push_back((uint8_t)(v >> 8));
    o.push_back((uint8_t)v);
}
void chunk(std::vector<uint8_t>& o, const char* type, const uint8_t* data, size_t len)
{
    be32(o, (uint32_t)len);
    size_t start = o.size();
    o.insert(o.end(), type, type + 4);
    o.insert(o.end(), data, data + len);
    uint32_t crc = (uint32_t)crc32(0L, o.data() + start, (uInt)(len + 4));
    be32(o, crc);
}

// PNG filter choice per row as stb_image_write does it (minimum sum of
// absolute filtered bytes over the five filters, PNG spec 9.2-9.4).
void filter_row(const uint8_t* cur, const uint8_t* up, int bytes, uint8_t* dst)
{
    static thread_local std::vector<uint8_t> tmp;
    tmp.resize((size_t)bytes);
    int best_sum = -1;
    for (int ft = 0; ft < 5; ++ft) {
        int sum = 0;
        for (int i = 0; i < bytes; ++i) {
            const int a = i >= 4 ? cur[i - 4] : 0, b = up ? up[i] : 0, c = (up && i >= 4) ? up[i - 4] : 0;
            int pred = 0;
            switch (ft) {
                case 1: pred = a; break;
                case 2: pred = b; break;
                case 3: pred = (a + b) >> 1; break;
                case 4: {
                    const int pp = a + b - c, pa = abs(pp - a), pb = abs(pp - b), pc = abs(pp - c);
                    pred = (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
                    break;
                }
                default: break;
            }
            const uint8_t v = (uint8_t)(cur[i] - pred);
            tmp[(size_t)i] = v;
            sum += (int8_t)v < 0 ? -(int8_t)v : (int8_t)v;
        }
        if (best_sum < 0 || sum < best_sum) {
            best_sum = sum;
            dst[0] = (uint8_t)ft;
            memcpy(dst + 1, tmp.data(), (size_t)bytes);
        }
    }
}

}  // namespace

// stbi_write_png + flip (main.cpp:341-342), parallel:
// rows are filtered and deflated in strips on host threads; each strip is a
// raw deflate stream ending on a byte boundary (Z_SYNC_FLUSH; the last one
// Z_FINISH) primed with the previous strip's last 32 KiB as its dictionary, so
// the strips concatenate into ONE zlib stream (adler32 combined) -- a single
// ordinary IDAT any decoder reads.  Threads: TMPT_PNG_THREADS (1 = sequential).
int write_png(const char* path, const uint8_t* rgba, int w, int h)
{
    const size_t stride = (size_t)w * 4 + 1;
    std::vector<uint8_t> raw((size_t)h * stride);
    // file row r (top-down) = image row h-1-r (bottom-up, stbi flip)
    auto img_row = [&](int r) { return rgba + (size_t)(h - 1 - r) * (size_t)w * 4; };
    const int nthreads = host_threads("TMPT_PNG_THREADS");
    const int strip_rows = std::max(1, env_int("TMPT_PNG_STRIP", 64));
    const int nstrips = std::max(1, (h + strip_rows - 1) / strip_rows);
    std::vector<std::vector<uint8_t>> zs((size_t)nstrips);
    std::vector<uLong> adl((size_t)nstrips);
    std::atomic<int> next{0};
    std::atomic<bool> failed{false};
    auto work = [&]() {
        for (int k; (k = next.fetch_add(1)) < nstrips;) {
            const int r0 = k * strip_rows, r1 = std::min(h, r0 + strip_rows);
            for (int r = r0; r < r1; ++r)
                filter_row(img_row(r), r > 0 ? img_row(r - 1) : nullptr, w * 4, &raw[(size_t)r * stride]);
            const uint8_t* src = &raw[(size_t)r0 * stride];
            const size_t n = (size_t)(r1 - r0) * stride;
            adl[(size_t)k] = adler32(adler32(0L, Z_NULL, 0), src, (uInt)n);
            z_stream zs_{};
            if (deflateInit2(&zs_, 6, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) {
                failed = true;
                continue;
            }
            if (k > 0) {
                // dictionary = the last 32 KiB of the previous strip's filtered rows;
                // another thread may be writing those into `raw`, so filter them here
                const int need = (int)((32768 + stride - 1) / stride);
                const int p0 = std::max(0, r0 - std::min(strip_rows, need));
                std::vector<uint8_t> prev((size_t)(r0 - p0) * stride);
                for (int r = p0; r < r0; ++r)
                    filter_row(img_row(r), r > 0 ? img_row(r - 1) : nullptr, w * 4,
                               &prev[(size_t)(r - p0) * stride]);
                const size_t dn = std::min<size_t>(prev.size(), 32768);
                deflateSetDictionary(&zs_, prev.data() + prev.size() - dn, (uInt)dn);
            }
            std::vector<uint8_t>& out = zs[(size_t)k];
            out.resize(deflateBound(&zs_, (uLong)n) + 16);
            zs_.next_in = const_cast<Bytef*>(src);
            zs_.avail_in = (uInt)n;
            zs_.next_out = out.data();
            zs_.avail_out = (uInt)out.size();
            const int rc = deflate(&zs_, k == nstrips - 1 ? Z_FINISH : Z_SYNC_FLUSH);
            if ((k == nstrips - 1 && rc != Z_STREAM_END) || (k < nstrips - 1 && rc != Z_OK)) failed = true;
            out.resize(out.size() - zs_.avail_out);
            deflateEnd(&zs_);
        }
    };
    {
        std::vector<std::thread> pool;
        const int nt = std::min(nthreads, nstrips);
        for (int t = 1; t < nt; ++t) pool.emplace_back(work);
        work();
        for (auto& t : pool) t.join();
    }
    if (failed) {
        set_error("png: deflate failed");
        return -1;
    }
    std::vector<uint8_t> z = {0x78, 0x9C};  // zlib header: deflate, 32 KiB window, default level
    uLong ad = adl[0];
    for (int k = 0; k < nstrips; ++k) {
        z.insert(z.end(), zs[(size_t)k].begin(), zs[(size_t)k].end());
        if (k > 0) {
            const int r0 = k * strip_rows, r1 = std::min(h, r0 + strip_rows);
            ad = adler32_combine(ad, adl[(size_t)k], (z_off_t)((size_t)(r1 - r0) * stride));
        }
    }
    be32(z, (uint32_t)ad);
    const uLongf zlen = (uLongf)z.size();
    std::vector<uint8_t> out = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1A, '\n'};
    uint8_t ihdr[13];
    ihdr[0] = (uint8_t)(w >> 24); ihdr[1] = (uint8_t)(w >> 16); ihdr[2] = (uint8_t)(w >> 8); ihdr[3] = (uint8_t)w;
    ihdr[4] = (uint8_t)(h >> 24); ihdr[5] = (uint8_t)(h >> 16); ihdr[6] = (uint8_t)(h >> 8); ihdr[7] = (uint8_t)h;
    ihdr[8] = 8;   // bit depth
    ihdr[9] = 6;   // RGBA
    ihdr[10] = 0; ihdr[11] = 0; ihdr[12] = 0;
    chunk(out, "IHDR", ihdr, 13);
    chunk(out, "IDAT", z.data(), zlen);
    chunk(out, "IEND", nullptr, 0);
    FILE* f = fopen(path, "wb");
    if (!f) {
        set_error(std::string("cannot write '") + path + "'");
        return -1;
    }
    size_t put = fwrite(out.data(), 1, out.size(), f);
    fclose(f);
    if (put != out.size()) {
        set_error("png: short write");
        return -1;
    }
    return 0;
}

}  // namespace tmpt
