// gsr_ply.cpp — host PLY loading into the SoA scene arrays, and the seeded
// synthetic scene writers (SURVEY.md 8d, config 5 spec in DESIGN.md).
//
// Two modes:
//   reference (flags 0): restates loadGaussianCudaFromPly (misc.cu:13-134) and
//     storeGaussianFromProperty (gaussians.cpp:17-30) exactly — the first
//     "format" line, the first "element vertex" line, then every "property"
//     line up to end_header (of any element) counts as a vertex property and is
//     read as a 4-byte float whatever its declared type; only
//     binary_little_endian 1.0; "nxx" (sic) is the first normal; f_rest_j kept
//     for j < 24.
//   typed (GSR_PLY_TYPED): the hardened reader — declared
//     property types (int8..float64 and their aliases), ascii /
//     binary_little_endian / binary_big_endian, elements before and after the
//     vertex element skipped properly (list properties included), "nx" or "nxx".
// Both map the same names to the same arrays and apply the same activations,
// plus the Spacetime-Gaussian 4D properties (trbf_center, trbf_scale,
// motion_0..8) into arrays 38..48 when the caller asks for 49 arrays, and
// (GSR_PLY_SH3, 59 arrays) all 45 f_rest mapped channel-major -> sh[3k + c].
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <fstream>
#include <random>
#include <sstream>
#include <string>
#include <vector>

#include "gsr.h"
#include "gsr_internal.h"

using gsr::set_error;

namespace {

enum Slot { S_X, S_Y, S_Z, S_NORMAL, S_DC, S_REST, S_OPACITY, S_SCALE, S_ROT, S_TCENTER, S_TSCALE, S_MOTION, S_SKIP };
enum Type { T_I8, T_U8, T_I16, T_U16, T_I32, T_U32, T_F32, T_F64, T_BAD };

struct Prop {
    Slot slot = S_SKIP;
    int index = 0;
    Type type = T_F32;
    bool is_list = false;
    Type count_type = T_U8;
};

struct Element {
    std::string name;
    int64_t count = 0;
    std::vector<Prop> props;
};

struct PlyHeader {
    std::string format;
    int64_t n = -1;
    std::vector<Prop> props;          // vertex properties (reference mode: every property line)
    std::vector<Element> elements;    // typed mode
    int vertex_element = -1;
};

Type parse_type(const std::string& s) {
    if (s == "char" || s == "int8") return T_I8;
    if (s == "uchar" || s == "uint8") return T_U8;
    if (s == "short" || s == "int16") return T_I16;
    if (s == "ushort" || s == "uint16") return T_U16;
    if (s == "int" || s == "int32") return T_I32;
    if (s == "uint" || s == "uint32") return T_U32;
    if (s == "float" || s == "float32") return T_F32;
    if (s == "double" || s == "float64") return T_F64;
    return T_BAD;
}

int type_size(Type t) {
    switch (t) {
    case T_I8: case T_U8: return 1;
    case T_I16: case T_U16: return 2;
    case T_I32: case T_U32: case T_F32: return 4;
    case T_F64: return 8;
    default: return 0;
    }
}

// Name -> (slot, index); the reference's map (misc.cu:60-90) plus "nx" in typed
// mode and the 4D names.
Prop slot_for(const std::string& name, bool typed, bool sh3) {
    Prop p;
    if (name == "x") p.slot = S_X;
    else if (name == "y") p.slot = S_Y;
    else if (name == "z") p.slot = S_Z;
    else if (name == "nxx" || (typed && name == "nx")) p.slot = S_NORMAL, p.index = 0;   // sic, misc.cu:68
    else if (name == "ny") p.slot = S_NORMAL, p.index = 1;
    else if (name == "nz") p.slot = S_NORMAL, p.index = 2;
    else if (name == "f_dc_0") p.slot = S_DC, p.index = 0;
    else if (name == "f_dc_1") p.slot = S_DC, p.index = 1;
    else if (name == "f_dc_2") p.slot = S_DC, p.index = 2;
    else if (name.rfind("f_rest_", 0) == 0) {
        const int idx = std::atoi(name.c_str() + 7);
        if (idx >= 0 && idx < (sh3 ? 45 : 24)) p.slot = S_REST, p.index = idx;   // misc.cu:76 (24)
    } else if (name == "opacity") p.slot = S_OPACITY;
    else if (name.rfind("scale_", 0) == 0) {
        const int idx = std::atoi(name.c_str() + 6);
        if (idx >= 0 && idx < 3) p.slot = S_SCALE, p.index = idx;
    } else if (name.rfind("rot_", 0) == 0) {
        const int idx = std::atoi(name.c_str() + 4);
        if (idx >= 0 && idx < 4) p.slot = S_ROT, p.index = idx;
    } else if (name == "trbf_center") p.slot = S_TCENTER;
    else if (name == "trbf_scale") p.slot = S_TSCALE;
    else if (name.rfind("motion_", 0) == 0) {
        const int idx = std::atoi(name.c_str() + 7);
        if (idx >= 0 && idx < 9) p.slot = S_MOTION, p.index = idx;
    }
    return p;
}

bool starts(const std::string& s, const char* pre) { return s.compare(0, std::strlen(pre), pre) == 0; }

// misc.cu:21-58 as written: first "format ", first "element vertex ", then every
// "property" line until end_header.
int parse_header_reference(std::ifstream& file, PlyHeader& h, bool sh3) {
    std::string line;
    while (std::getline(file, line))
        if (starts(line, "format ")) {
            h.format = line.substr(7);
            break;
        }
    bool found = false;
    while (std::getline(file, line))
        if (starts(line, "element vertex ")) {
            found = true;
            break;
        }
    if (!found) return set_error(GSR_E_FORMAT, "PLY: no 'element vertex' line");
    try {
        h.n = std::stoll(line.substr(15));
    } catch (...) {
        return set_error(GSR_E_FORMAT, "PLY: bad vertex count '%s'", line.c_str());
    }
    if (h.n < 0 || h.n > INT32_MAX) return set_error(GSR_E_FORMAT, "PLY: vertex count out of range");
    while (std::getline(file, line)) {
        if (line == "end_header") break;
        if (!starts(line, "property ")) continue;
        std::istringstream iss(line.substr(9));
        std::string type, name;
        iss >> type >> name;
        h.props.push_back(slot_for(name, false, sh3));   // type ignored: read as float (misc.cu:103)
    }
    if (h.format != "binary_little_endian 1.0")
        return set_error(GSR_E_FORMAT, "Unsupported PLY format: %s", h.format.c_str());
    return GSR_OK;
}

int parse_header_typed(std::ifstream& file, PlyHeader& h, bool sh3) {
    std::string line;
    if (!std::getline(file, line) || line.compare(0, 3, "ply") != 0) return set_error(GSR_E_FORMAT, "PLY: missing magic");
    bool done = false;
    while (std::getline(file, line)) {
        if (!line.empty() && line.back() == '\r') line.pop_back();
        std::istringstream iss(line);
        std::string kw;
        iss >> kw;
        if (kw == "format") {
            std::string f, v;
            iss >> f >> v;
            h.format = f;
        } else if (kw == "element") {
            Element e;
            iss >> e.name >> e.count;
            if (!iss || e.count < 0) return set_error(GSR_E_FORMAT, "PLY: bad element line '%s'", line.c_str());
            h.elements.push_back(e);
        } else if (kw == "property") {
            if (h.elements.empty()) return set_error(GSR_E_FORMAT, "PLY: property before element");
            std::string t1;
            iss >> t1;
            Prop p;
            std::string name;
            if (t1 == "list") {
                std::string ct, it;
                iss >> ct >> it >> name;
                p.is_list = true;
                p.count_type = parse_type(ct);
                p.type = parse_type(it);
                if (p.count_type == T_BAD || p.type == T_BAD || p.count_type == T_F32 || p.count_type == T_F64)
                    return set_error(GSR_E_FORMAT, "PLY: bad list property '%s' (integer count type required)",
                                     line.c_str());
            } else {
                iss >> name;
                p.type = parse_type(t1);
                if (p.type == T_BAD) return set_error(GSR_E_FORMAT, "PLY: bad property type '%s'", t1.c_str());
                const Prop s = slot_for(name, true, sh3);
                p.slot = s.slot;
                p.index = s.index;
            }
            h.elements.back().props.push_back(p);
        } else if (kw == "end_header") {
            done = true;
            break;
        }   // comment / obj_info / unknown keywords: ignored
    }
    if (!done) return set_error(GSR_E_FORMAT, "PLY: no end_header");
    for (size_t i = 0; i < h.elements.size(); i++)
        if (h.elements[i].name == "vertex") {
            h.vertex_element = (int)i;
            break;
        }
    if (h.vertex_element < 0) return set_error(GSR_E_FORMAT, "PLY: no 'element vertex' line");
    h.n = h.elements[h.vertex_element].count;
    if (h.n > INT32_MAX) return set_error(GSR_E_FORMAT, "PLY: vertex count out of range");
    if (h.format != "binary_little_endian" && h.format != "binary_big_endian" && h.format != "ascii")
        return set_error(GSR_E_FORMAT, "Unsupported PLY format: %s", h.format.c_str());
    return GSR_OK;
}

// storeGaussianFromProperty (gaussians.cpp:17-30) into SoA arrays; 4D
// properties only when the caller's table has them.
inline void store(const Prop& p, float* soa, int narrays, int64_t n, int64_t i, float v) {
    switch (p.slot) {
    case S_X: soa[GSR_A_X * n + i] = v; break;
    case S_Y: soa[GSR_A_Y * n + i] = v; break;
    case S_Z: soa[GSR_A_Z * n + i] = v; break;
    case S_DC: soa[(GSR_A_SH0 + p.index) * n + i] = v; break;
    case S_REST:
        if (narrays == GSR_SCENE_SH3_NARRAYS)   // channel-major f_rest -> coefficient-major sh[3k + c]
            soa[(GSR_A_SH0 + 3 * (1 + p.index % 15) + p.index / 15) * n + i] = v;
        else
            soa[(GSR_A_SH0 + 3 + p.index) * n + i] = v;
        break;
    case S_OPACITY: soa[GSR_A_OPACITY * n + i] = 1.0f / (1.0f + std::exp(-v)); break;   // sigmoid<float>
    case S_SCALE: soa[(GSR_A_SCALE0 + p.index) * n + i] = (float)::exp((double)v); break; // ::exp(double)
    case S_ROT: soa[(GSR_A_ROT0 + p.index) * n + i] = v; break;
    case S_TCENTER: if (narrays == GSR_SCENE4D_NARRAYS) soa[GSR_A_TCENTER * n + i] = v; break;
    case S_TSCALE:
        if (narrays == GSR_SCENE4D_NARRAYS) soa[GSR_A_TSCALE * n + i] = (float)::exp((double)v);
        break;
    case S_MOTION: if (narrays == GSR_SCENE4D_NARRAYS) soa[(GSR_A_MOTION0 + p.index) * n + i] = v; break;
    default: break;   // normals and skipped properties are not used by the render path
    }
}

// A decoded value as the float the SoA arrays hold: out-of-range magnitudes become
// +-inf and NaN stays NaN (IEEE conversion, without the undefined behaviour of a
// double -> float cast out of range).
float to_float(double d) {
    if (d > (double)FLT_MAX) return INFINITY;
    if (d < -(double)FLT_MAX) return -INFINITY;
    return (float)d;
}

// List lengths beyond this are malformed (a PLY face has a handful of indices).
constexpr int64_t kMaxListLen = int64_t(1) << 24;

// Bytes the rows of the vertex element need, when they can be known from the header
// (binary formats, every element before and including it fixed-size); -1 otherwise.
int64_t vertex_data_bytes(const PlyHeader& h, bool typed) {
    if (!typed) return (int64_t)h.props.size() * 4 * h.n;
    if (h.format == "ascii") return -1;
    int64_t total = 0;
    for (int ei = 0; ei <= h.vertex_element; ei++) {
        int64_t row = 0;
        for (const Prop& p : h.elements[ei].props) {
            if (p.is_list) return -1;
            row += type_size(p.type);
        }
        const int64_t cnt = h.elements[ei].count;
        if (row && cnt > (INT64_MAX - total) / row) return INT64_MAX;
        total += row * cnt;
    }
    return total;
}

template <typename T>
T load_as(const unsigned char* b, bool swap) {
    unsigned char tmp[sizeof(T)];
    std::memcpy(tmp, b, sizeof(T));
    if (swap) std::reverse(tmp, tmp + sizeof(T));
    T v;
    std::memcpy(&v, tmp, sizeof(T));
    return v;
}

double decode(Type t, const unsigned char* b, bool swap) {
    switch (t) {
    case T_I8: return (double)(int8_t)b[0];
    case T_U8: return (double)b[0];
    case T_I16: return (double)load_as<int16_t>(b, swap);
    case T_U16: return (double)load_as<uint16_t>(b, swap);
    case T_I32: return (double)load_as<int32_t>(b, swap);
    case T_U32: return (double)load_as<uint32_t>(b, swap);
    case T_F32: return (double)load_as<float>(b, swap);
    case T_F64: return load_as<double>(b, swap);
    default: return 0.0;
    }
}

bool has_4d(const std::vector<Prop>& props) {
    for (const Prop& p : props)
        if (p.slot == S_TCENTER) return true;
    return false;
}

int read_reference(std::ifstream& file, const PlyHeader& h, float* soa, int narrays, const char* path) {
    const int64_t n = h.n;
    const size_t np = h.props.size();
    std::vector<float> buf;
    const int64_t chunk = 65536;
    for (int64_t i0 = 0; i0 < n; i0 += chunk) {
        const int64_t m = std::min(chunk, n - i0);
        buf.resize((size_t)m * np);
        if (np && !file.read(reinterpret_cast<char*>(buf.data()), (std::streamsize)(buf.size() * sizeof(float))))
            return set_error(GSR_E_IO, "PLY: truncated data in %s", path);
        for (int64_t r = 0; r < m; r++)
            for (size_t p = 0; p < np; p++) store(h.props[p], soa, narrays, n, i0 + r, buf[(size_t)r * np + p]);
    }
    return GSR_OK;
}

// Skip (or read, for the vertex element) the rows of every element in order.
int read_typed(std::ifstream& file, const PlyHeader& h, float* soa, int narrays, const char* path) {
    const int64_t n = h.n;
    if (h.format == "ascii") {
        std::string line;
        for (size_t ei = 0; ei < h.elements.size(); ei++) {
            const Element& e = h.elements[ei];
            const bool vert = (int)ei == h.vertex_element;
            for (int64_t r = 0; r < e.count; r++) {
                if (!std::getline(file, line)) return set_error(GSR_E_IO, "PLY: truncated ascii data in %s", path);
                std::istringstream iss(line);
                for (const Prop& p : e.props) {
                    if (p.is_list) {
                        double cnt = -1;
                        if (!(iss >> cnt) || !(cnt >= 0 && cnt <= (double)kMaxListLen))   // NaN included
                            return set_error(GSR_E_FORMAT, "PLY: bad ascii list length in row %lld", (long long)r);
                        for (int64_t k = 0; k < (int64_t)cnt; k++) {
                            double d;
                            if (!(iss >> d))
                                return set_error(GSR_E_FORMAT, "PLY: short ascii list in row %lld", (long long)r);
                        }
                        continue;
                    }
                    double d = 0;
                    if (!(iss >> d)) return set_error(GSR_E_FORMAT, "PLY: bad ascii row %lld", (long long)r);
                    if (vert) store(p, soa, narrays, n, r, to_float(d));
                }
            }
            if (vert) return GSR_OK;   // rows after the vertex element are not needed
        }
        return GSR_OK;
    }
    const bool swap = h.format == "binary_big_endian";   // hosts here are little-endian
    for (size_t ei = 0; ei < h.elements.size(); ei++) {
        const Element& e = h.elements[ei];
        const bool vert = (int)ei == h.vertex_element;
        bool fixed = true;
        size_t row = 0;
        for (const Prop& p : e.props) {
            if (p.is_list) fixed = false;
            row += (size_t)type_size(p.type);
        }
        if (fixed && row == 0) {   // an element without properties has no data
            if (vert) return GSR_OK;
            continue;
        }
        if (fixed) {
            const int64_t chunk = std::max<int64_t>(1, (int64_t)((8u << 20) / std::max<size_t>(row, 1)));
            std::vector<unsigned char> buf;
            for (int64_t i0 = 0; i0 < e.count; i0 += chunk) {
                const int64_t m = std::min(chunk, e.count - i0);
                buf.resize((size_t)m * row);
                if (row && !file.read(reinterpret_cast<char*>(buf.data()), (std::streamsize)buf.size()))
                    return set_error(GSR_E_IO, "PLY: truncated data in %s", path);
                if (!vert) continue;
                for (int64_t r = 0; r < m; r++) {
                    const unsigned char* b = buf.data() + (size_t)r * row;
                    for (const Prop& p : e.props) {
                        if (p.slot != S_SKIP) store(p, soa, narrays, n, i0 + r, to_float(decode(p.type, b, swap)));
                        b += type_size(p.type);
                    }
                }
            }
        } else {
            for (int64_t r = 0; r < e.count; r++)
                for (const Prop& p : e.props) {
                    unsigned char b[8];
                    if (p.is_list) {
                        if (!file.read(reinterpret_cast<char*>(b), type_size(p.count_type)))
                            return set_error(GSR_E_IO, "PLY: truncated data in %s", path);
                        const double dc = decode(p.count_type, b, swap);   // an integer type (header check)
                        if (dc < 0 || dc > (double)kMaxListLen)
                            return set_error(GSR_E_FORMAT, "PLY: bad list length %.0f", dc);
                        const int64_t cnt = (int64_t)dc;
                        file.seekg((std::streamoff)(cnt * type_size(p.type)), std::ios::cur);
                        continue;
                    }
                    if (!file.read(reinterpret_cast<char*>(b), type_size(p.type)))
                        return set_error(GSR_E_IO, "PLY: truncated data in %s", path);
                    if (vert && p.slot != S_SKIP) store(p, soa, narrays, n, r, to_float(decode(p.type, b, swap)));
                }
        }
        if (vert) return GSR_OK;
    }
    return GSR_OK;
}

}  // namespace

extern "C" int gsr_ply_read_host_ex(const char* path, float* soa, int narrays, int64_t capacity, int64_t* n_out,
                                    int flags, int* is_4d) {
    if (!path || !n_out) return set_error(GSR_E_ARG, "gsr_ply_read_host: null argument");
    const bool sh3 = (flags & GSR_PLY_SH3) != 0;
    if (sh3 ? narrays != GSR_SCENE_SH3_NARRAYS : (narrays != GSR_SCENE_NARRAYS && narrays != GSR_SCENE4D_NARRAYS))
        return set_error(GSR_E_ARG, "gsr_ply_read_host: narrays must be %d or %d (%d with GSR_PLY_SH3)",
                         GSR_SCENE_NARRAYS, GSR_SCENE4D_NARRAYS, GSR_SCENE_SH3_NARRAYS);
    std::ifstream file(path, std::ios::binary);
    if (!file.is_open()) return set_error(GSR_E_IO, "Failed to open file: %s", path);
    PlyHeader h;
    const bool typed = (flags & GSR_PLY_TYPED) != 0;
    int rc = typed ? parse_header_typed(file, h, sh3) : parse_header_reference(file, h, sh3);
    if (h.n >= 0) *n_out = h.n;
    if (rc) return rc;
    if (is_4d) *is_4d = has_4d(typed ? h.elements[h.vertex_element].props : h.props) ? 1 : 0;
    // a header whose vertex count the data cannot hold is refused before the caller
    // sizes buffers from it (counts come from the file: hostile or truncated headers)
    const int64_t need = vertex_data_bytes(h, typed);
    if (need >= 0) {
        const std::streampos here = file.tellg();
        file.seekg(0, std::ios::end);
        const std::streamoff avail = file.tellg() - here;
        file.seekg(here);
        if (!file || need > (int64_t)avail)
            return set_error(GSR_E_IO, "PLY: %s holds %lld data bytes, its header needs %lld", path,
                             (long long)avail, (long long)need);
    }
    if (!soa || capacity < h.n) return GSR_OK;
    std::fill(soa, soa + (size_t)narrays * (size_t)h.n, 0.0f);   // Gaussian g{} (misc.cu:97)
    if (narrays == GSR_SCENE4D_NARRAYS)   // 4D defaults: static Gaussian (centre 0, scale 1, no motion)
        std::fill(soa + (size_t)GSR_A_TSCALE * (size_t)h.n, soa + (size_t)(GSR_A_TSCALE + 1) * (size_t)h.n, 1.0f);
    return typed ? read_typed(file, h, soa, narrays, path) : read_reference(file, h, soa, narrays, path);
}

extern "C" int gsr_ply_read_host(const char* path, float* soa, int64_t capacity, int64_t* n_out) {
    return gsr_ply_read_host_ex(path, soa, GSR_SCENE_NARRAYS, capacity, n_out, 0, nullptr);
}

// ------------------------------------------------------------------ synthetic scenes

namespace {

int write_synth(const char* path, int64_t n, uint64_t seed, bool four_d) {
    if (!path || n < 0 || n > INT32_MAX) return set_error(GSR_E_ARG, "gsr_synth_write_ply: bad argument");
    std::ofstream f(path, std::ios::binary);
    if (!f) return set_error(GSR_E_IO, "cannot write %s", path);
    f << "ply\nformat binary_little_endian 1.0\nelement vertex " << n << "\n";
    const char* base[] = {"x", "y", "z", "nx", "ny", "nz", "f_dc_0", "f_dc_1", "f_dc_2"};
    for (const char* b : base) f << "property float " << b << "\n";
    for (int r = 0; r < 45; r++) f << "property float f_rest_" << r << "\n";
    f << "property float opacity\n";
    for (int r = 0; r < 3; r++) f << "property float scale_" << r << "\n";
    for (int r = 0; r < 4; r++) f << "property float rot_" << r << "\n";
    if (four_d) {
        f << "property float trbf_center\nproperty float trbf_scale\n";
        for (int r = 0; r < 9; r++) f << "property float motion_" << r << "\n";
    }
    f << "end_header\n";
    const int nprop = four_d ? 73 : 62;
    std::mt19937_64 rng(seed);
    std::uniform_real_distribution<float> ux(-3.0f, 3.0f), uy(-1.7f, 1.7f), uz(-1.0f, 1.0f);
    std::normal_distribution<float> ndc(0.0f, 0.6f), nrest(0.0f, 0.15f), nrot(0.0f, 1.0f);
    std::uniform_real_distribution<float> uop(-1.0f, 3.0f), usc(-5.65f, -4.07f);
    // config 5: centre U(0,1), log temporal scale U(-3.5,-2), motion
    // N(0, 0.5) linear, N(0, 0.2) quadratic, N(0, 0.1) cubic (world units / unit time^k)
    std::uniform_real_distribution<float> utc(0.0f, 1.0f), uts(-3.5f, -2.0f);
    std::normal_distribution<float> nm1(0.0f, 0.5f), nm2(0.0f, 0.2f), nm3(0.0f, 0.1f);
    std::vector<float> row((size_t)nprop);
    std::vector<float> block;
    block.reserve((size_t)nprop * 4096);
    for (int64_t i = 0; i < n; i++) {
        int k = 0;
        row[k++] = ux(rng);
        row[k++] = uy(rng);
        row[k++] = uz(rng);
        row[k++] = 0.0f;
        row[k++] = 0.0f;
        row[k++] = 0.0f;
        for (int c = 0; c < 3; c++) row[k++] = ndc(rng);
        for (int c = 0; c < 45; c++) row[k++] = nrest(rng);
        row[k++] = uop(rng);
        for (int c = 0; c < 3; c++) row[k++] = usc(rng);
        for (int c = 0; c < 4; c++) row[k++] = nrot(rng);
        if (four_d) {
            row[k++] = utc(rng);
            row[k++] = uts(rng);
            for (int c = 0; c < 3; c++) row[k++] = nm1(rng);
            for (int c = 0; c < 3; c++) row[k++] = nm2(rng);
            for (int c = 0; c < 3; c++) row[k++] = nm3(rng);
        }
        block.insert(block.end(), row.begin(), row.end());
        if (block.size() >= (size_t)nprop * 4096) {
            f.write(reinterpret_cast<const char*>(block.data()), (std::streamsize)(block.size() * sizeof(float)));
            block.clear();
        }
    }
    f.write(reinterpret_cast<const char*>(block.data()), (std::streamsize)(block.size() * sizeof(float)));
    if (!f) return set_error(GSR_E_IO, "write failed: %s", path);
    return GSR_OK;
}

}  // namespace

extern "C" int gsr_synth_write_ply(const char* path, int64_t n, uint64_t seed) {
    return write_synth(path, n, seed, false);
}

extern "C" int gsr_synth_write_ply4d(const char* path, int64_t n, uint64_t seed) {
    return write_synth(path, n, seed, true);
}
