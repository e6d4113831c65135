// Checkpoints of the guiding distribution (.asdmm) -- host code over the C ABI.
//
// Reference: the integrator saves its accelerator once per render iteration,
// saveCheckpoint() -> sdmm::save_json(m_accelerator, "checkpoints/model_%05i.asdmm")
// (mitsuba/src/integrators/dmm/volpath_sdmm.cpp:117-126, called at :441); the
// single-mixture counterpart is jmm MixtureModel::save/load (dmm/jmm/
// mixture_model.h:315-326, fields serialised at :379-388).  sdmm-lib, which
// holds save_json, is absent from the snapshot, so its JSON schema is unknown:
// this file defines one that carries everything a resumed
// run needs -- the tree's node table, per trained leaf the mixture's canonical
// AND derived arrays (restored verbatim, so a reloaded mixture guides and steps
// bitwise like the saved one) and the stepwise-EM state (G, T, priors,
// iteration count: stepwise_tangent.h:181-210).
//
// Numbers: floats are written with 9 and doubles with 17 significant digits
// (both round-trip exactly through strtof / strtod); non-finite values, which
// JSON has no literal for, as the strings "NaN", "Infinity", "-Infinity".
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <string_view>
#include <vector>

#include "../../include/sdmm_gpu.h"

namespace sdmm_detail {
int set_error(int code, const char* msg);   // sdmm_api.cpp
}

namespace {

constexpr const char* kFormat = "sdmm-amd.asdmm";
constexpr const char* kFormat4 = "sdmm-amd.sdmm4";   // a learned BSDF (sdmm_learned4_*)
constexpr int kVersion = 1;
constexpr int kScalars = 9;

int err(int code, const std::string& msg) { return sdmm_detail::set_error(code, msg.c_str()); }

// ---- writer ----------------------------------------------------------------
struct Writer {
    std::string s;
    void raw(const char* t) { s += t; }
    void key(const char* k) { s += '"'; s += k; s += "\":"; }
    void nonfinite(double v) { s += std::isnan(v) ? "\"NaN\"" : (v > 0 ? "\"Infinity\"" : "\"-Infinity\""); }
    void f32(float v) {
        if (!std::isfinite(v)) return nonfinite(v);
        char b[32];
        std::snprintf(b, sizeof b, "%.9g", (double)v);
        s += b;
    }
    void f64(double v) {
        if (!std::isfinite(v)) return nonfinite(v);
        char b[40];
        std::snprintf(b, sizeof b, "%.17g", v);
        s += b;
    }
    void i64(long long v) { s += std::to_string(v); }
    template <class T, class F>
    void array(const T* a, size_t n, F put) {
        s += '[';
        for (size_t i = 0; i < n; ++i) {
            if (i) s += ',';
            put(a[i]);
        }
        s += ']';
    }
    void farr(const char* k, const float* a, size_t n) { key(k); array(a, n, [&](float v) { f32(v); }); s += ','; }
    void darr(const char* k, const double* a, size_t n) { key(k); array(a, n, [&](double v) { f64(v); }); s += ','; }
    void iarr(const char* k, const int32_t* a, size_t n) { key(k); array(a, n, [&](int32_t v) { i64(v); }); s += ','; }
    void close_obj() {   // drop a trailing comma
        if (!s.empty() && s.back() == ',') s.pop_back();
        s += '}';
    }
};

// One mixture's field table: name, floats per component (the order of
// sdmm_params_out).
struct Field { const char* name; int width; };
const Field kParamFields[] = {{"weights", 1}, {"cdf", 1}, {"mean", 6}, {"cov", 25}, {"to", 9},
                              {"cholL", 25}, {"cholLInv", 25}, {"detInv", 1}, {"muPremult", 6},
                              {"condCov", 4}, {"margL", 9}, {"margDetInv", 1}, {"condL", 4},
                              {"condLInv", 4}, {"condDetInv", 1}};
constexpr int kNumParamFields = sizeof(kParamFields) / sizeof(kParamFields[0]);

float** param_slot(sdmm_params_out& o, int i) {
    float** slots[kNumParamFields] = {&o.weights, &o.cdf, &o.mean, &o.cov, &o.to, &o.cholL, &o.cholLInv,
                                      &o.detInv, &o.muPremult, &o.condCov, &o.margL, &o.margDetInv,
                                      &o.condL, &o.condLInv, &o.condDetInv};
    return slots[i];
}

struct MixImage {   // host image of one sdmm_mix
    int K = 0;
    sdmm_em_params ep{};
    std::vector<float> f[kNumParamFields];
    std::vector<int32_t> valid;
    float normalization = 1.0f;
    std::vector<double> scalars, T, sgW, sgM, sgC;
    std::vector<float> bpriors, bdepth;

    void size(int k) {
        K = k;
        for (int i = 0; i < kNumParamFields; ++i) f[i].assign((size_t)K * kParamFields[i].width, 0.0f);
        valid.assign((size_t)K, 0);
        scalars.assign(kScalars, 0.0);
        T.assign((size_t)K, 0.0); sgW.assign((size_t)K, 0.0);
        sgM.assign(5 * (size_t)K, 0.0); sgC.assign(25 * (size_t)K, 0.0);
        bpriors.assign(25 * (size_t)K, 0.0f); bdepth.assign(9 * (size_t)K, 0.0f);
    }
    sdmm_params_out view() {
        sdmm_params_out o{};
        for (int i = 0; i < kNumParamFields; ++i) *param_slot(o, i) = f[i].data();
        o.valid = valid.data();
        o.normalization = &normalization;
        return o;
    }
};

int fetch(const sdmm_mix* m, MixImage& im) {
    im.size(sdmm_num_components(m));
    int r = sdmm_get_em_params(m, &im.ep);
    if (r) return r;
    sdmm_params_out o = im.view();
    if ((r = sdmm_get_params(m, &o))) return r;
    return sdmm_get_state(m, im.scalars.data(), im.T.data(), im.sgW.data(), im.sgM.data(), im.sgC.data(),
                          im.bpriors.data(), im.bdepth.data());
}

void write_mix(Writer& w, const MixImage& im) {
    const size_t K = (size_t)im.K;
    w.raw("{");
    w.key("K"); w.i64(im.K); w.raw(",");
    w.key("em_params"); w.raw("{");
    w.key("alpha"); w.f32(im.ep.alpha); w.raw(",");
    w.farr("bprior", im.ep.bprior, 5);
    w.key("ni_prior_minus_one"); w.f32(im.ep.ni_prior_minus_one); w.raw(",");
    w.key("epsilon"); w.f64(im.ep.epsilon); w.raw(",");
    w.key("decrease_prior"); w.i64(im.ep.decrease_prior);
    w.raw("},");
    for (int i = 0; i < kNumParamFields; ++i) w.farr(kParamFields[i].name, im.f[i].data(), im.f[i].size());
    w.iarr("valid", im.valid.data(), K);
    w.key("normalization"); w.f32(im.normalization); w.raw(",");
    w.key("state"); w.raw("{");
    w.darr("scalars", im.scalars.data(), kScalars);
    w.darr("T", im.T.data(), K);
    w.darr("sgW", im.sgW.data(), K);
    w.darr("sgM", im.sgM.data(), 5 * K);
    w.darr("sgC", im.sgC.data(), 25 * K);
    w.farr("bpriors", im.bpriors.data(), 25 * K);
    w.farr("bdepth", im.bdepth.data(), 9 * K);
    w.close_obj();
    w.raw("}");
}

int write_file(const char* path, const std::string& s) {
    FILE* fp = std::fopen(path, "wb");
    if (!fp) return err(SDMM_E_INVALID, std::string("cannot open ") + path + " for writing");
    const size_t n = std::fwrite(s.data(), 1, s.size(), fp);
    const int c = std::fclose(fp);
    if (n != s.size() || c != 0) return err(SDMM_E_INVALID, std::string("short write to ") + path);
    return SDMM_OK;
}

// ---- reader: a small JSON DOM over the file text.  Scalars are views into
// the text (converted when their type is known); an array of numbers (or of
// the non-finite strings) is kept as one vector of views, 16 B per element --
// the per-leaf parameter arrays are almost all of a checkpoint.
struct Value {
    enum Kind { Null, Bool, Num, Str, Arr, Obj } kind = Null;
    std::string_view text;                  // Num / Str
    bool b = false;
    std::vector<Value> arr;                 // Arr of objects / arrays
    std::vector<std::string_view> nums;     // Arr of numbers / strings (views; strings unquoted)
    std::vector<bool> num_is_str;
    std::map<std::string, Value, std::less<>> obj;
    const Value* get(const char* k) const {
        if (kind != Obj) return nullptr;
        auto it = obj.find(std::string_view(k));
        return it != obj.end() ? &it->second : nullptr;
    }
    size_t size() const { return arr.empty() ? nums.size() : arr.size(); }
};

struct Parser {
    const char* p;
    const char* end;
    std::string error;
    int depth = 0;

    void ws() { while (p < end && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p; }
    bool fail(const char* what) { if (error.empty()) error = what; return false; }
    bool lit(const char* w) {
        const size_t n = std::strlen(w);
        if ((size_t)(end - p) < n || std::strncmp(p, w, n) != 0) return fail("bad literal");
        p += n;
        return true;
    }
    // the writer never escapes: a string is the text between its quotes (an
    // escape is rejected rather than mis-read)
    bool str(std::string_view& out) {
        if (p >= end || *p != '"') return fail("expected string");
        const char* s = ++p;
        while (p < end && *p != '"') {
            if (*p == '\\') return fail("escaped strings are not used by this format");
            ++p;
        }
        if (p >= end) return fail("unterminated string");
        out = std::string_view(s, (size_t)(p - s));
        ++p;
        return true;
    }
    bool number(std::string_view& out) {
        const char* s = p;
        while (p < end && (std::strchr("+-.eE", *p) || (*p >= '0' && *p <= '9'))) ++p;
        if (p == s) return fail("unexpected character");
        out = std::string_view(s, (size_t)(p - s));
        return true;
    }
    bool array(Value& v) {
        v.kind = Value::Arr;
        ++p; ws();
        if (p < end && *p == ']') { ++p; return true; }
        const bool scalars = p < end && *p != '{' && *p != '[';
        for (;;) {
            ws();
            if (scalars) {
                std::string_view t;
                const bool is_str = p < end && *p == '"';
                if (!(is_str ? str(t) : number(t))) return false;
                v.nums.push_back(t);
                v.num_is_str.push_back(is_str);
            } else {
                v.arr.emplace_back();
                if (!value(v.arr.back())) return false;
            }
            ws();
            if (p < end && *p == ',') { ++p; continue; }
            if (p < end && *p == ']') { ++p; return true; }
            return fail("expected ',' or ']'");
        }
    }
    bool value(Value& v) {
        if (++depth > 64) return fail("nesting too deep");
        ws();
        if (p >= end) return fail("unexpected end");
        bool ok = true;
        if (*p == '{') {
            v.kind = Value::Obj;
            ++p; ws();
            if (p < end && *p == '}') { ++p; --depth; return true; }
            while (ok) {
                ws();
                std::string_view k;
                if (!str(k)) return false;
                ws();
                if (p >= end || *p != ':') return fail("expected ':'");
                ++p;
                if (!value(v.obj[std::string(k)])) return false;
                ws();
                if (p < end && *p == ',') { ++p; continue; }
                if (p < end && *p == '}') { ++p; break; }
                return fail("expected ',' or '}'");
            }
        } else if (*p == '[') {
            ok = array(v);
        } else if (*p == '"') {
            v.kind = Value::Str;
            ok = str(v.text);
        } else if (*p == 't') { v.kind = Value::Bool; v.b = true; ok = lit("true"); }
        else if (*p == 'f') { v.kind = Value::Bool; ok = lit("false"); }
        else if (*p == 'n') { ok = lit("null"); }
        else {
            v.kind = Value::Num;
            ok = number(v.text);
        }
        --depth;
        return ok;
    }
};

// text -> number through a NUL-terminated copy (numbers are short)
bool text_f64(std::string_view t, bool is_str, double& out) {
    if (is_str) {
        if (t == "NaN") { out = std::nan(""); return true; }
        if (t == "Infinity") { out = HUGE_VAL; return true; }
        if (t == "-Infinity") { out = -HUGE_VAL; return true; }
        return false;
    }
    char b[64];
    if (t.empty() || t.size() >= sizeof b) return false;
    std::memcpy(b, t.data(), t.size());
    b[t.size()] = 0;
    char* e = nullptr;
    out = std::strtod(b, &e);
    return e == b + t.size();
}
bool text_f32(std::string_view t, bool is_str, float& out) {
    if (is_str) {
        double d;
        if (!text_f64(t, true, d)) return false;
        out = (float)d;
        return true;
    }
    char b[64];
    if (t.empty() || t.size() >= sizeof b) return false;
    std::memcpy(b, t.data(), t.size());
    b[t.size()] = 0;
    char* e = nullptr;
    out = std::strtof(b, &e);   // nearest float of the 9-digit text: exact round trip
    return e == b + t.size();
}
bool text_int(std::string_view t, bool is_str, long long& out) {
    if (is_str) return false;
    char b[32];
    if (t.empty() || t.size() >= sizeof b) return false;
    std::memcpy(b, t.data(), t.size());
    b[t.size()] = 0;
    char* e = nullptr;
    errno = 0;
    out = std::strtoll(b, &e, 10);
    return e == b + t.size() && errno == 0;
}
bool num_f64(const Value& v, double& out) {
    return (v.kind == Value::Num || v.kind == Value::Str) && text_f64(v.text, v.kind == Value::Str, out);
}
bool num_f32(const Value& v, float& out) {
    return (v.kind == Value::Num || v.kind == Value::Str) && text_f32(v.text, v.kind == Value::Str, out);
}
bool num_int(const Value& v, long long& out) { return v.kind == Value::Num && text_int(v.text, false, out); }

template <class T, class F>
bool read_array(const Value* v, std::vector<T>& out, size_t n, F conv) {
    if (!v || v->kind != Value::Arr || !v->arr.empty() || v->nums.size() != n) return false;
    out.resize(n);
    for (size_t i = 0; i < n; ++i)
        if (!conv(v->nums[i], v->num_is_str[i], out[i])) return false;
    return true;
}
bool farr(const Value& o, const char* k, std::vector<float>& out, size_t n) {
    return read_array(o.get(k), out, n, text_f32);
}
bool darr(const Value& o, const char* k, std::vector<double>& out, size_t n) {
    return read_array(o.get(k), out, n, text_f64);
}
bool iarr(const Value& o, const char* k, std::vector<int32_t>& out, size_t n) {
    return read_array(o.get(k), out, n, [](std::string_view t, bool is_str, int32_t& x) {
        long long l;
        if (!text_int(t, is_str, l) || l < INT32_MIN || l > INT32_MAX) return false;
        x = (int32_t)l;
        return true;
    });
}

int read_file(const char* path, std::string& s, Value& root, const char* format = kFormat) {
    FILE* fp = std::fopen(path, "rb");
    if (!fp) return err(SDMM_E_INVALID, std::string("cannot open ") + path);
    char buf[1 << 16];
    size_t n;
    while ((n = std::fread(buf, 1, sizeof buf, fp)) > 0) s.append(buf, n);
    std::fclose(fp);
    Parser ps{s.data(), s.data() + s.size(), {}};
    if (!ps.value(root)) return err(SDMM_E_INVALID, std::string(path) + ": JSON parse error: " + ps.error);
    ps.ws();
    if (ps.p != ps.end) return err(SDMM_E_INVALID, std::string(path) + ": trailing data after JSON");
    const Value* f = root.get("format");
    const Value* ver = root.get("version");
    long long vv = 0;
    if (!f || f->kind != Value::Str || f->text != format || !ver || !num_int(*ver, vv) || vv != kVersion)
        return err(SDMM_E_INVALID, std::string(path) + ": not an " + format + " file (format/version)");
    return SDMM_OK;
}

int parse_mix(const Value& o, MixImage& im, const std::string& where) {
    const Value* kv = o.get("K");
    long long K = 0;
    if (!kv || !num_int(*kv, K) || K < 1 || K > 512) return err(SDMM_E_INVALID, where + ": bad K");
    im.size((int)K);
    const Value* ep = o.get("em_params");
    std::vector<float> bp, tmp;
    std::vector<double> eps;
    long long dec = 0;
    if (!ep || !farr(*ep, "bprior", bp, 5) || !ep->get("alpha") || !num_f32(*ep->get("alpha"), im.ep.alpha) ||
        !ep->get("ni_prior_minus_one") || !num_f32(*ep->get("ni_prior_minus_one"), im.ep.ni_prior_minus_one) ||
        !ep->get("epsilon") || !num_f64(*ep->get("epsilon"), im.ep.epsilon) || !ep->get("decrease_prior") ||
        !num_int(*ep->get("decrease_prior"), dec))
        return err(SDMM_E_INVALID, where + ": bad em_params");
    for (int i = 0; i < 5; ++i) im.ep.bprior[i] = bp[(size_t)i];
    im.ep.decrease_prior = (int)dec;
    const size_t k = (size_t)K;
    for (int i = 0; i < kNumParamFields; ++i)
        if (!farr(o, kParamFields[i].name, im.f[i], k * kParamFields[i].width))
            return err(SDMM_E_INVALID, where + ": bad field " + kParamFields[i].name);
    if (!iarr(o, "valid", im.valid, k) || !o.get("normalization") || !num_f32(*o.get("normalization"), im.normalization))
        return err(SDMM_E_INVALID, where + ": bad valid/normalization");
    const Value* st = o.get("state");
    if (!st || !darr(*st, "scalars", im.scalars, kScalars) || !darr(*st, "T", im.T, k) ||
        !darr(*st, "sgW", im.sgW, k) || !darr(*st, "sgM", im.sgM, 5 * k) || !darr(*st, "sgC", im.sgC, 25 * k) ||
        !farr(*st, "bpriors", im.bpriors, 25 * k) || !farr(*st, "bdepth", im.bdepth, 9 * k))
        return err(SDMM_E_INVALID, where + ": bad stepwise state");
    return SDMM_OK;
}

int instantiate(MixImage& im, int device, sdmm_mix** out) {
    *out = nullptr;
    sdmm_mix* m = nullptr;
    int r = sdmm_create(im.K, &im.ep, device, &m);
    if (r) return r;
    sdmm_params_out o = im.view();
    if ((r = sdmm_restore_params(m, &o)) ||
        (r = sdmm_set_state(m, im.scalars.data(), im.T.data(), im.sgW.data(), im.sgM.data(), im.sgC.data(),
                            im.bpriors.data(), im.bdepth.data()))) {
        sdmm_destroy(m);
        return r;
    }
    *out = m;
    return SDMM_OK;
}

}  // namespace

extern "C" {

int sdmm_mix_save_json(const sdmm_mix* m, const char* path) {
    if (!m || !path) return err(SDMM_E_INVALID, "invalid argument");
    MixImage im;
    int r = fetch(m, im);
    if (r) return r;
    Writer w;
    w.raw("{\"format\":\"");
    w.raw(kFormat);
    w.raw("\",\"version\":");
    w.i64(kVersion);
    w.raw(",\"mixture\":");
    write_mix(w, im);
    w.raw("}\n");
    return write_file(path, w.s);
}

int sdmm_mix_load_json(const char* path, int device, sdmm_mix** out) {
    if (!path || !out) return err(SDMM_E_INVALID, "invalid argument");
    *out = nullptr;
    std::string text;   // the values below are views into it
    Value root;
    int r = read_file(path, text, root);
    if (r) return r;
    const Value* mv = root.get("mixture");
    if (!mv || mv->kind != Value::Obj) return err(SDMM_E_INVALID, std::string(path) + ": no mixture");
    MixImage im;
    if ((r = parse_mix(*mv, im, path))) return r;
    return instantiate(im, device, out);
}

int sdmm_save_json(const sdmm_stree* t, const sdmm_mix* const* node_mix, const char* path) {
    if (!t || !path) return err(SDMM_E_INVALID, "invalid argument");
    const int n = sdmm_stree_num_nodes(t);
    std::vector<float> aabb(6 * (size_t)n);
    std::vector<int32_t> child(2 * (size_t)n), axis((size_t)n);
    int r = sdmm_stree_get_nodes(t, aabb.data(), child.data(), axis.data());
    if (r) return r;
    Writer w;
    w.raw("{\"format\":\"");
    w.raw(kFormat);
    w.raw("\",\"version\":");
    w.i64(kVersion);
    w.raw(",\"num_nodes\":");
    w.i64(n);
    w.raw(",\"nodes\":{");
    w.farr("aabb", aabb.data(), aabb.size());
    w.iarr("child", child.data(), child.size());
    w.iarr("axis", axis.data(), axis.size());
    w.close_obj();
    w.raw(",\"mixtures\":[");
    bool first = true;
    for (int i = 0; node_mix && i < n; ++i) {
        const sdmm_mix* m = node_mix[i];
        if (!m) continue;
        MixImage im;
        if ((r = fetch(m, im))) return r;
        if (!first) w.raw(",");
        first = false;
        w.raw("{\"node\":");
        w.i64(i);
        w.raw(",\"mixture\":");
        write_mix(w, im);
        w.raw("}");
    }
    w.raw("]}\n");
    return write_file(path, w.s);
}

int sdmm_load_json(const char* path, int device, sdmm_stree** tree_out, sdmm_mix** node_mix_out, int cap,
                   int* num_nodes_out) {
    if (!path) return err(SDMM_E_INVALID, "invalid argument");
    if (tree_out) *tree_out = nullptr;
    std::string text;   // the values below are views into it
    Value root;
    int r = read_file(path, text, root);
    if (r) return r;
    long long n = 0;
    const Value* nv = root.get("num_nodes");
    if (!nv || !num_int(*nv, n) || n < 1 || n > (1 << 26)) return err(SDMM_E_INVALID, std::string(path) + ": bad num_nodes");
    if (num_nodes_out) *num_nodes_out = (int)n;
    if (!tree_out) return SDMM_OK;   // size query
    if (!node_mix_out || cap < n) return err(SDMM_E_INVALID, "node_mix_out must hold num_nodes handles");
    const Value* nodes = root.get("nodes");
    std::vector<float> aabb;
    std::vector<int32_t> child, axis;
    const size_t un = (size_t)n;
    if (!nodes || !farr(*nodes, "aabb", aabb, 6 * un) || !iarr(*nodes, "child", child, 2 * un) ||
        !iarr(*nodes, "axis", axis, un))
        return err(SDMM_E_INVALID, std::string(path) + ": bad node table");
    const Value* mixes = root.get("mixtures");
    if (!mixes || mixes->kind != Value::Arr) return err(SDMM_E_INVALID, std::string(path) + ": no mixtures array");
    // parse everything before creating device objects: a bad file allocates nothing
    std::vector<std::pair<int, std::unique_ptr<MixImage>>> images;
    if (!mixes->nums.empty()) return err(SDMM_E_INVALID, std::string(path) + ": mixtures must be objects");
    std::vector<char> seen(un, 0);
    for (size_t j = 0; j < mixes->arr.size(); ++j) {
        const Value& e = mixes->arr[j];
        long long node = -1;
        const std::string where = std::string(path) + ": mixtures[" + std::to_string(j) + "]";
        if (!e.get("node") || !num_int(*e.get("node"), node) || node < 0 || node >= n)
            return err(SDMM_E_INVALID, where + ": bad node id");
        if (seen[(size_t)node]) return err(SDMM_E_INVALID, where + ": duplicate node id");
        seen[(size_t)node] = 1;
        const Value* mv = e.get("mixture");
        if (!mv) return err(SDMM_E_INVALID, where + ": no mixture");
        std::unique_ptr<MixImage> im(new MixImage());
        if ((r = parse_mix(*mv, *im, where))) return r;
        images.emplace_back((int)node, std::move(im));
    }
    // the tree: any root box (set_nodes replaces the table wholesale)
    const float lo[3] = {0, 0, 0}, hi[3] = {1, 1, 1};
    sdmm_stree* t = nullptr;
    if ((r = sdmm_stree_create(lo, hi, device, &t))) return r;
    if ((r = sdmm_stree_set_nodes(t, (int)n, aabb.data(), child.data(), axis.data()))) {
        sdmm_stree_destroy(t);
        return r;
    }
    for (int i = 0; i < n; ++i) node_mix_out[i] = nullptr;
    for (auto& pr : images) {
        if ((r = instantiate(*pr.second, device, &node_mix_out[pr.first]))) {
            for (int i = 0; i < n; ++i) { sdmm_destroy(node_mix_out[i]); node_mix_out[i] = nullptr; }
            sdmm_stree_destroy(t);
            return r;
        }
    }
    *tree_out = t;
    return SDMM_OK;
}


// ---------------------------------------------------------------------------
// OpenEXR (scanline, NO_COMPRESSION, FLOAT channels B G R) -- the per-pass
// image dumps of SDMMWorkResult::dumpIndividual (sdmm_wr.cpp:115-146).
// A learned BSDF (sdmm_learned_bsdf4): {"format": "sdmm-amd.sdmm4",
// "version": 1, "M": M, "weights": [M], "means": [5M], "covs": [16M]} --
// floats written with 9 significant digits (exact round trip).
int sdmm_learned4_save_json(const sdmm_learned_bsdf4* m, const char* path) {
    if (!m || !path || m->M < 1 || m->M > 8 || !m->weights || !m->means || !m->covs)
        return err(SDMM_E_INVALID, "sdmm_learned4_save_json: invalid argument");
    Writer w;
    w.raw("{\"format\":\"");
    w.raw(kFormat4);
    w.raw("\",\"version\":");
    w.i64(kVersion);
    w.raw(",\"M\":");
    w.i64(m->M);
    w.raw(",");
    w.farr("weights", m->weights, (size_t)m->M);
    w.farr("means", m->means, 5 * (size_t)m->M);
    w.farr("covs", m->covs, 16 * (size_t)m->M);
    w.close_obj();
    w.raw("\n");
    FILE* fp = std::fopen(path, "wb");
    if (!fp) return err(SDMM_E_INVALID, std::string("cannot write ") + path);
    const bool ok = std::fwrite(w.s.data(), 1, w.s.size(), fp) == w.s.size();
    if (std::fclose(fp) != 0 || !ok) return err(SDMM_E_INVALID, std::string("write failed: ") + path);
    return SDMM_OK;
}

int sdmm_learned4_load_json(const char* path, int cap, int* M_out, float* weights, float* means, float* covs) {
    if (!path || !M_out || cap < 0 || (cap > 0 && (!weights || !means || !covs)))
        return err(SDMM_E_INVALID, "sdmm_learned4_load_json: invalid argument");
    std::string text;
    Value root;
    int r = read_file(path, text, root, kFormat4);
    if (r) return r;
    const Value* mv = root.get("M");
    long long M = 0;
    if (!mv || !num_int(*mv, M) || M < 1 || M > 8) return err(SDMM_E_INVALID, std::string(path) + ": bad M");
    std::vector<float> w, mu, c;
    if (!farr(root, "weights", w, (size_t)M) || !farr(root, "means", mu, 5 * (size_t)M) ||
        !farr(root, "covs", c, 16 * (size_t)M))
        return err(SDMM_E_INVALID, std::string(path) + ": weights / means / covs missing or of the wrong size");
    *M_out = (int)M;
    if (cap == 0) return SDMM_OK;
    if (cap < M) return err(SDMM_E_INVALID, std::string(path) + ": cap smaller than M");
    std::memcpy(weights, w.data(), sizeof(float) * w.size());
    std::memcpy(means, mu.data(), sizeof(float) * mu.size());
    std::memcpy(covs, c.data(), sizeof(float) * c.size());
    return SDMM_OK;
}

int sdmm_write_exr(const char* path, int width, int height, const float* rgb, int spp, int iteration, float time) {
    if (!path || !rgb || width < 1 || height < 1) return err(SDMM_E_INVALID, "sdmm_write_exr: invalid argument");
    std::string h;
    auto put_u32 = [&](uint32_t v) { for (int i = 0; i < 4; ++i) h.push_back((char)((v >> (8 * i)) & 0xFF)); };
    auto put_f32 = [&](float f) { uint32_t v; std::memcpy(&v, &f, 4); put_u32(v); };
    auto put_str = [&](const char* t) { h.append(t); h.push_back('\0'); };
    auto attr = [&](const char* name, const char* type, const std::string& value) {
        put_str(name);
        put_str(type);
        put_u32((uint32_t)value.size());
        h += value;
    };
    put_u32(20000630u);   // magic
    put_u32(2u);          // version 2, single-part scanline
    {
        std::string ch;
        for (const char* c : {"B", "G", "R"}) {   // channel list, alphabetical
            ch.append(c);
            ch.push_back('\0');
            const int32_t v[4] = {2, 0, 1, 1};   // FLOAT, pLinear 0 + 3 reserved bytes, xSampling, ySampling
            ch.append((const char*)&v[0], 4);
            ch.append((const char*)&v[1], 4);
            ch.append((const char*)&v[2], 4);
            ch.append((const char*)&v[3], 4);
        }
        ch.push_back('\0');
        attr("channels", "chlist", ch);
    }
    attr("compression", "compression", std::string(1, '\0'));
    const int32_t box[4] = {0, 0, width - 1, height - 1};
    attr("dataWindow", "box2i", std::string((const char*)box, 16));
    attr("displayWindow", "box2i", std::string((const char*)box, 16));
    attr("lineOrder", "lineOrder", std::string(1, '\0'));
    {
        const float one = 1.0f, zero[2] = {0.0f, 0.0f};
        attr("pixelAspectRatio", "float", std::string((const char*)&one, 4));
        attr("screenWindowCenter", "v2f", std::string((const char*)zero, 8));
        attr("screenWindowWidth", "float", std::string((const char*)&one, 4));
    }
    {
        const int32_t a = spp, b = iteration;
        attr("spp", "int", std::string((const char*)&a, 4));
        attr("iteration", "int", std::string((const char*)&b, 4));
        attr("time", "float", std::string((const char*)&time, 4));
    }
    h.push_back('\0');   // end of header
    (void)put_f32;
    const uint64_t line_bytes = 8 + 3 * 4 * (uint64_t)width;
    const uint64_t first = (uint64_t)h.size() + 8 * (uint64_t)height;
    FILE* f = std::fopen(path, "wb");
    if (!f) return err(SDMM_E_INVALID, std::string("sdmm_write_exr: cannot open ") + path);
    bool ok = std::fwrite(h.data(), 1, h.size(), f) == h.size();
    for (int y = 0; y < height && ok; ++y) {
        const uint64_t off = first + line_bytes * (uint64_t)y;
        ok = std::fwrite(&off, 8, 1, f) == 1;
    }
    const size_t plane = (size_t)width * (size_t)height;
    for (int y = 0; y < height && ok; ++y) {
        const int32_t hdr[2] = {y, (int32_t)(3 * 4 * width)};
        ok = std::fwrite(hdr, 4, 2, f) == 2;
        for (int c = 2; c >= 0 && ok; --c)   // B, G, R
            ok = std::fwrite(rgb + (size_t)c * plane + (size_t)y * width, 4, (size_t)width, f) == (size_t)width;
    }
    ok = (std::fclose(f) == 0) && ok;
    return ok ? SDMM_OK : err(SDMM_E_INVALID, std::string("sdmm_write_exr: write failed: ") + path);
}

}  // extern "C"
