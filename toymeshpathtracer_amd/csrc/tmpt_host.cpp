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

#include <cmath>
#include <string>
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

}  // namespace

int load_obj(const char* path, std::vector<float>& tris, f3& bmin, f3& bmax)
{
    FILE* f = fopen(path, "rb");
    if (!f) {
        set_error(std::string("cannot open '") + (path ? path : "") + "'");
        return -1;
    }
    std::string text;
    char buf[1 << 16];
    size_t got;
    while ((got = fread(buf, 1, sizeof(buf), f)) > 0) text.append(buf, got);
    fclose(f);

    std::vector<float> pos;      // xyz per vertex
    std::vector<int32_t> faces;  // 3 position indices per triangle (0-based)
    const char* p = text.data();
    const char* end = p + text.size();
    while (p < end) {
        const char* eol = (const char*)memchr(p, '\n', (size_t)(end - p));
        const char* le = eol ? eol : end;
        Cursor c{p, le};
        if (le - p >= 2 && p[0] == 'v' && p[1] == ' ') {
            c.p += 2;
            float x = read_float(c), y = read_float(c), z = read_float(c);
            pos.push_back(x);
            pos.push_back(y);
            pos.push_back(z);
        } else if (le - p >= 2 && p[0] == 'f' && p[1] == ' ') {
            c.p += 2;
            const int nv = (int)(pos.size() / 3);
            int fan0 = 0, prev = 0, k = 0;
            while (c.p < c.end) {
                int vi = read_face_vertex(c);
                if (vi == 0) break;
                int idx = vi >= 0 ? vi - 1 : nv + vi;  // objparser.cpp:29-32
                if (k == 0) fan0 = idx;
                else if (k >= 2) {
                    faces.push_back(fan0);
                    faces.push_back(prev);
                    faces.push_back(idx);
                }
                prev = idx;
                ++k;
            }
        }
        p = le + 1;
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
}  // namespace

int write_png(const char* path, const uint8_t* rgba, int w, int h)
{
    // rows are written top-down from the bottom-up image (stbi flip, main.cpp:341)
    std::vector<uint8_t> raw((size_t)h * ((size_t)w * 4 + 1));
    for (int r = 0; r < h; ++r) {
        uint8_t* dst = &raw[(size_t)r * ((size_t)w * 4 + 1)];
        dst[0] = 0;  // filter: none
        memcpy(dst + 1, rgba + (size_t)(h - 1 - r) * w * 4, (size_t)w * 4);
    }
    uLongf zlen = compressBound((uLong)raw.size());
    std::vector<uint8_t> z(zlen);
    if (compress2(z.data(), &zlen, raw.data(), (uLong)raw.size(), 6) != Z_OK) {
        set_error("png: deflate failed");
        return -1;
    }
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
