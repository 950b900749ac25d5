// kmerhip_napi.cc — thin N-API addon over the libkmerhip C-ABI
// (include/kmer_api.h).  All counting runs on the GPU inside napi_async_work
// (libuv pool); the completion callback hands packed results back to JS,
// where kmers.js builds the Map in the reference's insertion order.
//
// JS surface (used by kmers.js only):
//   open(k, prefixBuffer, step, device, flags, maxKeys, batchBytes, devices[]) -> handle
//     (devices: >= 2 HIP ordinals -> a multi-GPU group context, kmer_params.ndev)
//   countFile(handle, path, cb(err, {keys, offsets, counts, lines}), progress(done, total)?)
//   indexKeys(keysBuffer, offsetsFloat64Array, n, cap) -> Int32Array (KmerMap index)
//   countBuffer(handle, buffer, cb(err, {...}), progress(done, total)?)
//     (progress: called on the JS thread after each input batch, kmer_params.progress)
//   close(handle)
//   version() -> string
// Template matching (include/kmer_match.h; used by kmerfinder.js), synchronous:
//   dbOpen(k, keysBuffer, startsFloat64Array, device) -> db
//   dbInfo(db) -> {k, templates, distinct, entries};  dbClose(db)
//   matchOpen(db, keysBuffer, offsetsFloat64Array, countsFloat64Array) -> match
//   matchTemplates(match, order) -> {tmpl: Uint32Array, u: Float64Array, t: Float64Array}
//   matchTemplateKmers(match, tmpl) -> Uint32Array (round-1 query indices of tmpl)
//   matchWinner(match) -> {tmpl (-1: none), uscore, tscore, hits, firstU, firstT}
//   matchRemove(match, tmpl) -> hits left;  matchRemoved(match) -> Uint8Array
//   matchClose(match)
#include <node_api.h>

#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/kmer_api.h"
#include "../../include/kmer_match.h"

namespace {

#define NAPI_CALL(env, call)                                                    \
    do {                                                                        \
        if ((call) != napi_ok) {                                                \
            napi_throw_error((env), nullptr, "N-API call failed: " #call);     \
            return nullptr;                                                     \
        }                                                                       \
    } while (0)

struct Handle {
    kmer_ctx *ctx = nullptr;
    bool busy = false;
    bool close_pending = false;   // close() while a call was in flight: closed when it completes
    napi_threadsafe_function tsfn = nullptr;   // the in-flight call's progress callback (or none)
};

// kmer_params.progress of every context: runs on the counting thread (libuv
// pool), hands (done, total) to the JS thread through the call's
// thread-safe function
void progress_trampoline(void *user, uint64_t done, uint64_t total) {
    Handle *h = static_cast<Handle *>(user);
    if (!h->tsfn) return;
    double *d = new double[2]{(double)done, (double)total};
    if (napi_call_threadsafe_function(h->tsfn, d, napi_tsfn_nonblocking) != napi_ok) delete[] d;
}

void progress_call_js(napi_env env, napi_value js_cb, void *, void *data) {
    double *d = static_cast<double *>(data);
    if (env && js_cb) {
        napi_value undef, args[2];
        napi_get_undefined(env, &undef);
        napi_create_double(env, d[0], &args[0]);
        napi_create_double(env, d[1], &args[1]);
        napi_call_function(env, undef, js_cb, 2, args, nullptr);
    }
    delete[] d;
}

struct Work {
    napi_async_work work = nullptr;
    napi_ref cb = nullptr;
    napi_ref keep = nullptr;   // keeps the input Buffer alive
    napi_ref href = nullptr;   // keeps the handle's external alive while Execute uses it
    Handle *h = nullptr;
    std::string path;
    const uint8_t *bytes = nullptr;
    size_t len = 0;
    bool is_file = false;
    kmer_status st = KMER_OK;
    std::string err;
    kmer_result *res = nullptr;
};

void finalize_handle(napi_env, void *data, void *) {
    Handle *h = static_cast<Handle *>(data);
    if (h->ctx) kmer_close(h->ctx);
    delete h;
}

Handle *get_handle(napi_env env, napi_value v) {
    void *p = nullptr;
    if (napi_get_value_external(env, v, &p) != napi_ok || !p) {
        napi_throw_type_error(env, nullptr, "invalid kmerhip handle");
        return nullptr;
    }
    return static_cast<Handle *>(p);
}

uint32_t get_u32(napi_env env, napi_value v, uint32_t dflt) {
    napi_valuetype t;
    napi_typeof(env, v, &t);
    if (t != napi_number) return dflt;
    double d = 0;
    napi_get_value_double(env, v, &d);
    return d < 0 ? 0u : (uint32_t)d;
}

napi_value Open(napi_env env, napi_callback_info info) {
    size_t argc = 8;
    napi_value argv[8];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    if (argc < 3) {
        napi_throw_type_error(env, nullptr, "open(k, prefix, step, ...)");
        return nullptr;
    }
    void *pdata = nullptr;
    size_t plen = 0;
    bool isbuf = false;
    napi_is_buffer(env, argv[1], &isbuf);
    if (!isbuf) {
        napi_throw_type_error(env, nullptr, "prefix must be a Buffer (latin1)");
        return nullptr;
    }
    NAPI_CALL(env, napi_get_buffer_info(env, argv[1], &pdata, &plen));
    kmer_params p;
    memset(&p, 0, sizeof(p));
    p.k = get_u32(env, argv[0], 16);
    p.prefix = (const uint8_t *)pdata;
    p.prefix_len = (uint32_t)plen;
    p.step = get_u32(env, argv[2], 1);
    p.device = argc > 3 ? (int32_t)get_u32(env, argv[3], 0) : 0;
    p.flags = argc > 4 ? get_u32(env, argv[4], 0) : 0;
    if (argc > 5) {
        double d = 0;
        if (napi_get_value_double(env, argv[5], &d) == napi_ok && d > 0) p.max_keys = (uint64_t)d;
    }
    if (argc > 6) {
        double d = 0;
        if (napi_get_value_double(env, argv[6], &d) == napi_ok && d > 0) p.batch_bytes = (uint64_t)d;
    }
    std::vector<int32_t> devs;
    if (argc > 7) {                      // devices: an array of HIP ordinals -> multi-GPU group
        bool arr = false;
        napi_is_array(env, argv[7], &arr);
        if (arr) {
            uint32_t n = 0;
            napi_get_array_length(env, argv[7], &n);
            for (uint32_t i = 0; i < n; ++i) {
                napi_value e;
                napi_get_element(env, argv[7], i, &e);
                devs.push_back((int32_t)get_u32(env, e, 0));
            }
        }
    }
    if (devs.size() > 1) {
        p.ndev = (uint32_t)devs.size();
        p.devices = devs.data();
    }
    Handle *h = new Handle();
    p.progress = progress_trampoline;
    p.progress_user = h;
    kmer_status st = kmer_open(&p, &h->ctx);
    if (st != KMER_OK) {
        delete h;
        std::string msg = std::string("kmer_open: ") + kmer_status_string(st);
        napi_value err, code, m;
        napi_create_string_utf8(env, msg.c_str(), NAPI_AUTO_LENGTH, &m);
        napi_create_error(env, nullptr, m, &err);
        napi_create_int32(env, (int)st, &code);
        napi_set_named_property(env, err, "status", code);
        napi_throw(env, err);
        return nullptr;
    }
    napi_value ext;
    NAPI_CALL(env, napi_create_external(env, h, finalize_handle, nullptr, &ext));
    return ext;
}

void Execute(napi_env, void *data) {
    Work *w = static_cast<Work *>(data);
    if (w->is_file)
        w->st = kmer_count_file(w->h->ctx, w->path.c_str(), &w->res);
    else
        w->st = kmer_count_buffer(w->h->ctx, w->bytes, w->len, &w->res);
    if (w->st != KMER_OK) w->err = std::string(kmer_status_string(w->st)) + ": " + kmer_last_error(w->h->ctx);
}

napi_value make_f64_array(napi_env env, const uint64_t *src, size_t n) {
    napi_value ab, ta;
    void *data = nullptr;
    napi_create_arraybuffer(env, n * sizeof(double), &data, &ab);
    double *d = static_cast<double *>(data);
    for (size_t i = 0; i < n; ++i) d[i] = (double)src[i];
    napi_create_typedarray(env, napi_float64_array, n, ab, 0, &ta);
    return ta;
}

void Complete(napi_env env, napi_status, void *data) {
    Work *w = static_cast<Work *>(data);
    w->h->busy = false;
    if (w->h->tsfn) {                 // (progress calls already queued are still delivered)
        napi_release_threadsafe_function(w->h->tsfn, napi_tsfn_release);
        w->h->tsfn = nullptr;
    }
    if (w->h->close_pending && w->h->ctx) {
        kmer_close(w->h->ctx);
        w->h->ctx = nullptr;
    }
    napi_value cb, undef, args[2];
    napi_get_reference_value(env, w->cb, &cb);
    napi_get_undefined(env, &undef);
    if (w->st != KMER_OK) {
        napi_value m, code;
        napi_create_string_utf8(env, w->err.c_str(), NAPI_AUTO_LENGTH, &m);
        napi_create_error(env, nullptr, m, &args[0]);
        napi_create_int32(env, (int)w->st, &code);
        napi_set_named_property(env, args[0], "status", code);
        args[1] = undef;
    } else {
        const char *keys = nullptr;
        const uint64_t *offs = nullptr, *cnts = nullptr;
        kmer_result_arrays(w->res, &keys, &offs, &cnts);
        const uint64_t n = kmer_result_size(w->res);
        napi_value obj, kb, lines;
        napi_create_object(env, &obj);
        void *copy = nullptr;
        napi_create_buffer_copy(env, (size_t)offs[n], n ? keys : "", &copy, &kb);
        napi_set_named_property(env, obj, "keys", kb);
        napi_set_named_property(env, obj, "offsets", make_f64_array(env, offs, n + 1));
        napi_set_named_property(env, obj, "counts", make_f64_array(env, cnts, n));
        napi_create_double(env, (double)kmer_result_lines(w->res), &lines);
        napi_set_named_property(env, obj, "lines", lines);
        args[0] = undef;
        args[1] = obj;
        kmer_result_free(w->res);
    }
    napi_call_function(env, undef, cb, 2, args, nullptr);
    napi_delete_reference(env, w->cb);
    if (w->keep) napi_delete_reference(env, w->keep);
    if (w->href) napi_delete_reference(env, w->href);
    napi_delete_async_work(env, w->work);
    delete w;
}

napi_value queue(napi_env env, Work *w, napi_value handle, napi_value cb, napi_value progress) {
    napi_value name;
    napi_create_string_utf8(env, "kmerhip.count", NAPI_AUTO_LENGTH, &name);
    if (progress) {
        napi_valuetype t;
        napi_typeof(env, progress, &t);
        if (t == napi_function)
            NAPI_CALL(env, napi_create_threadsafe_function(env, progress, nullptr, name, 0, 1, nullptr, nullptr, nullptr,
                                                           progress_call_js, &w->h->tsfn));
    }
    NAPI_CALL(env, napi_create_reference(env, cb, 1, &w->cb));
    NAPI_CALL(env, napi_create_reference(env, handle, 1, &w->href));
    NAPI_CALL(env, napi_create_async_work(env, nullptr, name, Execute, Complete, w, &w->work));
    w->h->busy = true;
    NAPI_CALL(env, napi_queue_async_work(env, w->work));
    napi_value undef;
    napi_get_undefined(env, &undef);
    return undef;
}

napi_value CountFile(napi_env env, napi_callback_info info) {
    size_t argc = 4;
    napi_value argv[4];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    Handle *h = get_handle(env, argv[0]);
    if (!h) return nullptr;
    if (h->busy || !h->ctx) {
        napi_throw_error(env, nullptr, h->ctx ? "kmerhip handle busy (one in-flight call per context)"
                                              : "kmerhip handle closed");
        return nullptr;
    }
    size_t n = 0;
    NAPI_CALL(env, napi_get_value_string_utf8(env, argv[1], nullptr, 0, &n));
    Work *w = new Work();
    w->path.resize(n + 1);
    NAPI_CALL(env, napi_get_value_string_utf8(env, argv[1], &w->path[0], n + 1, &n));
    w->path.resize(n);
    w->h = h;
    w->is_file = true;
    return queue(env, w, argv[0], argv[2], argc > 3 ? argv[3] : nullptr);
}

napi_value CountBuffer(napi_env env, napi_callback_info info) {
    size_t argc = 4;
    napi_value argv[4];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    Handle *h = get_handle(env, argv[0]);
    if (!h) return nullptr;
    if (h->busy || !h->ctx) {
        napi_throw_error(env, nullptr, h->ctx ? "kmerhip handle busy (one in-flight call per context)"
                                              : "kmerhip handle closed");
        return nullptr;
    }
    void *data = nullptr;
    size_t len = 0;
    NAPI_CALL(env, napi_get_buffer_info(env, argv[1], &data, &len));
    Work *w = new Work();
    w->h = h;
    w->bytes = (const uint8_t *)data;
    w->len = len;
    NAPI_CALL(env, napi_create_reference(env, argv[1], 1, &w->keep));
    return queue(env, w, argv[0], argv[2], argc > 3 ? argv[3] : nullptr);
}

napi_value Close(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    Handle *h = get_handle(env, argv[0]);
    if (!h) return nullptr;
    if (h->busy) {
        h->close_pending = true;          // closed by the in-flight call's completion
    } else if (h->ctx) {
        kmer_close(h->ctx);
        h->ctx = nullptr;
    }
    napi_value undef;
    napi_get_undefined(env, &undef);
    return undef;
}

napi_value Version(napi_env env, napi_callback_info) {
    napi_value v;
    napi_create_string_utf8(env, kmer_version(), NAPI_AUTO_LENGTH, &v);
    return v;
}


// ---------------------------------------------------------------------------
// template matching
// ---------------------------------------------------------------------------
struct DbHandle {
    kmer_db *db = nullptr;
};
struct MatchHandle {
    kmer_match *m = nullptr;
    napi_ref dbref = nullptr;     // the DB outlives the match
};

void finalize_db(napi_env, void *data, void *) {
    DbHandle *h = static_cast<DbHandle *>(data);
    // open matches keep the DB alive: kmer_db_close defers to the last match
    if (h->db) (void)kmer_db_close(h->db);
    delete h;
}

void finalize_match(napi_env env, void *data, void *) {
    MatchHandle *h = static_cast<MatchHandle *>(data);
    if (h->m) kmer_match_close(h->m);
    if (h->dbref) napi_delete_reference(env, h->dbref);
    delete h;
}

napi_value throw_match(napi_env env, kmer_status st, const char *what) {
    std::string msg = std::string(what) + ": " + kmer_status_string(st) + ": " + kmer_match_last_error();
    napi_value err, code, m;
    napi_create_string_utf8(env, msg.c_str(), NAPI_AUTO_LENGTH, &m);
    napi_create_error(env, nullptr, m, &err);
    napi_create_int32(env, (int)st, &code);
    napi_set_named_property(env, err, "status", code);
    napi_throw(env, err);
    return nullptr;
}

bool get_f64_as_u64(napi_env env, napi_value v, std::vector<uint64_t> &out) {
    bool is = false;
    napi_is_typedarray(env, v, &is);
    if (!is) return false;
    napi_typedarray_type t;
    size_t n = 0;
    void *data = nullptr;
    napi_value ab;
    size_t off = 0;
    if (napi_get_typedarray_info(env, v, &t, &n, &data, &ab, &off) != napi_ok || t != napi_float64_array) return false;
    const double *d = static_cast<const double *>(data);
    out.resize(n);
    for (size_t i = 0; i < n; ++i) out[i] = (uint64_t)d[i];
    return true;
}

template <typename T>
T *get_ext(napi_env env, napi_value v, const char *what) {
    void *p = nullptr;
    if (napi_get_value_external(env, v, &p) != napi_ok || !p) {
        napi_throw_type_error(env, nullptr, what);
        return nullptr;
    }
    return static_cast<T *>(p);
}

napi_value DbOpen(napi_env env, napi_callback_info info) {
    size_t argc = 4;
    napi_value argv[4];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    if (argc < 3) {
        napi_throw_type_error(env, nullptr, "dbOpen(k, keys, starts, device)");
        return nullptr;
    }
    const uint32_t k = get_u32(env, argv[0], 16);
    void *kd = nullptr;
    size_t klen = 0;
    bool isbuf = false;
    napi_is_buffer(env, argv[1], &isbuf);
    std::vector<uint64_t> starts;
    if (!isbuf || !get_f64_as_u64(env, argv[2], starts) || starts.empty()) {
        napi_throw_type_error(env, nullptr, "dbOpen: keys must be a Buffer, starts a Float64Array");
        return nullptr;
    }
    NAPI_CALL(env, napi_get_buffer_info(env, argv[1], &kd, &klen));
    const int32_t dev = argc > 3 ? (int32_t)get_u32(env, argv[3], 0) : 0;
    DbHandle *h = new DbHandle();
    kmer_status st = kmer_db_open(dev, k, (const char *)kd, starts.back(), starts.data(),
                                  (uint32_t)(starts.size() - 1), &h->db);
    if (st != KMER_OK) {
        delete h;
        return throw_match(env, st, "kmer_db_open");
    }
    if (k && (uint64_t)klen != starts.back() * k) {
        kmer_db_close(h->db);
        delete h;
        napi_throw_range_error(env, nullptr, "dbOpen: keys length != n * k");
        return nullptr;
    }
    napi_value ext;
    NAPI_CALL(env, napi_create_external(env, h, finalize_db, nullptr, &ext));
    return ext;
}

napi_value DbInfo(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    DbHandle *h = get_ext<DbHandle>(env, argv[0], "invalid db handle");
    if (!h) return nullptr;
    if (!h->db) {
        napi_throw_error(env, nullptr, "db closed");
        return nullptr;
    }
    uint32_t k = 0, nt = 0;
    uint64_t d = 0, e = 0;
    kmer_db_info(h->db, &k, &nt, &d, &e);
    napi_value o, v;
    napi_create_object(env, &o);
    napi_create_double(env, k, &v);
    napi_set_named_property(env, o, "k", v);
    napi_create_double(env, nt, &v);
    napi_set_named_property(env, o, "templates", v);
    napi_create_double(env, (double)d, &v);
    napi_set_named_property(env, o, "distinct", v);
    napi_create_double(env, (double)e, &v);
    napi_set_named_property(env, o, "entries", v);
    return o;
}

napi_value DbClose(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    DbHandle *h = get_ext<DbHandle>(env, argv[0], "invalid db handle");
    if (!h) return nullptr;
    // with matches of the DB still open, kmer_db_close defers the free to the
    // last kmer_match_close (matchOpen on this handle then throws 'db closed')
    if (h->db) kmer_db_close(h->db);
    h->db = nullptr;
    napi_value u;
    napi_get_undefined(env, &u);
    return u;
}

napi_value MatchOpen(napi_env env, napi_callback_info info) {
    size_t argc = 4;
    napi_value argv[4];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    if (argc < 4) {
        napi_throw_type_error(env, nullptr, "matchOpen(db, keys, offsets, counts)");
        return nullptr;
    }
    DbHandle *dh = get_ext<DbHandle>(env, argv[0], "invalid db handle");
    if (!dh) return nullptr;
    if (!dh->db) {
        napi_throw_error(env, nullptr, "db closed");
        return nullptr;
    }
    void *kd = nullptr;
    size_t klen = 0;
    bool isbuf = false;
    napi_is_buffer(env, argv[1], &isbuf);
    std::vector<uint64_t> offs, cnts;
    if (!isbuf || !get_f64_as_u64(env, argv[2], offs) || !get_f64_as_u64(env, argv[3], cnts) ||
        offs.size() < cnts.size() + 1) {
        napi_throw_type_error(env, nullptr, "matchOpen: keys Buffer, offsets / counts Float64Array");
        return nullptr;
    }
    NAPI_CALL(env, napi_get_buffer_info(env, argv[1], &kd, &klen));
    if (offs[cnts.size()] > klen) {
        napi_throw_range_error(env, nullptr, "matchOpen: offsets beyond the keys buffer");
        return nullptr;
    }
    MatchHandle *h = new MatchHandle();
    kmer_status st = kmer_match_open(dh->db, (const char *)kd, offs.data(), cnts.data(), cnts.size(), &h->m);
    if (st != KMER_OK) {
        delete h;
        return throw_match(env, st, "kmer_match_open");
    }
    napi_create_reference(env, argv[0], 1, &h->dbref);
    napi_value ext;
    NAPI_CALL(env, napi_create_external(env, h, finalize_match, nullptr, &ext));
    return ext;
}

MatchHandle *get_match(napi_env env, napi_value v) {
    MatchHandle *h = get_ext<MatchHandle>(env, v, "invalid match handle");
    if (h && !h->m) {
        napi_throw_error(env, nullptr, "match closed");
        return nullptr;
    }
    return h;
}

napi_value MatchTemplates(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    MatchHandle *h = get_match(env, argv[0]);
    if (!h) return nullptr;
    const uint32_t order = argc > 1 ? get_u32(env, argv[1], 0) : 0;
    uint32_t n = 0;
    kmer_status st = kmer_match_templates(h->m, order, 0, nullptr, nullptr, nullptr, &n);
    if (st != KMER_OK) return throw_match(env, st, "kmer_match_templates");
    std::vector<uint32_t> t(n);
    std::vector<uint64_t> u(n), s(n);
    st = kmer_match_templates(h->m, order, n, t.data(), u.data(), s.data(), &n);
    if (st != KMER_OK) return throw_match(env, st, "kmer_match_templates");
    napi_value o, ab, ta;
    napi_create_object(env, &o);
    void *data = nullptr;
    napi_create_arraybuffer(env, (size_t)n * 4, &data, &ab);
    if (n) memcpy(data, t.data(), (size_t)n * 4);
    napi_create_typedarray(env, napi_uint32_array, n, ab, 0, &ta);
    napi_set_named_property(env, o, "tmpl", ta);
    napi_set_named_property(env, o, "u", make_f64_array(env, u.data(), n));
    napi_set_named_property(env, o, "t", make_f64_array(env, s.data(), n));
    return o;
}

napi_value MatchTemplateKmers(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    MatchHandle *h = get_match(env, argv[0]);
    if (!h) return nullptr;
    const uint32_t t = get_u32(env, argv[1], 0);
    uint64_t n = 0;
    kmer_status st = kmer_match_template_kmers(h->m, t, 0, nullptr, &n);
    if (st != KMER_OK) return throw_match(env, st, "kmer_match_template_kmers");
    napi_value ab, ta;
    void *data = nullptr;
    napi_create_arraybuffer(env, (size_t)n * 4, &data, &ab);
    st = kmer_match_template_kmers(h->m, t, n, static_cast<uint32_t *>(data), &n);
    if (st != KMER_OK) return throw_match(env, st, "kmer_match_template_kmers");
    napi_create_typedarray(env, napi_uint32_array, (size_t)n, ab, 0, &ta);
    return ta;
}

napi_value MatchWinner(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    MatchHandle *h = get_match(env, argv[0]);
    if (!h) return nullptr;
    kmer_winner w;
    kmer_status st = kmer_match_winner(h->m, &w);
    if (st != KMER_OK) return throw_match(env, st, "kmer_match_winner");
    napi_value o, v;
    napi_create_object(env, &o);
    napi_create_double(env, w.tmpl == 0xFFFFFFFFu ? -1.0 : (double)w.tmpl, &v);
    napi_set_named_property(env, o, "tmpl", v);
    const std::pair<const char *, uint64_t> f[] = {{"uscore", w.uscore}, {"tscore", w.tscore}, {"hits", w.hits},
                                                   {"firstU", w.first_uscore}, {"firstT", w.first_tscore}};
    for (const auto &x : f) {
        napi_create_double(env, (double)x.second, &v);
        napi_set_named_property(env, o, x.first, v);
    }
    return o;
}

napi_value MatchRemove(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    MatchHandle *h = get_match(env, argv[0]);
    if (!h) return nullptr;
    uint64_t hits = 0;
    kmer_status st = kmer_match_remove(h->m, get_u32(env, argv[1], 0), &hits);
    if (st != KMER_OK) return throw_match(env, st, "kmer_match_remove");
    napi_value v;
    napi_create_double(env, (double)hits, &v);
    return v;
}

napi_value MatchRemoved(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    MatchHandle *h = get_match(env, argv[0]);
    if (!h) return nullptr;
    const uint32_t n = argc > 1 ? get_u32(env, argv[1], 0) : 0;     // the query size
    napi_value ab, ta;
    void *data = nullptr;
    napi_create_arraybuffer(env, n, &data, &ab);
    kmer_status st = kmer_match_removed(h->m, static_cast<uint8_t *>(data));
    if (st != KMER_OK) return throw_match(env, st, "kmer_match_removed");
    napi_create_typedarray(env, napi_uint8_array, n, ab, 0, &ta);
    return ta;
}

napi_value MatchClose(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    MatchHandle *h = get_ext<MatchHandle>(env, argv[0], "invalid match handle");
    if (!h) return nullptr;
    if (h->m) kmer_match_close(h->m);
    h->m = nullptr;
    napi_value u;
    napi_get_undefined(env, &u);
    return u;
}

// indexKeys(keys Buffer, offsets Float64Array, n, cap) -> Int32Array(cap): the
// KmerMap's key -> packed index table (kmer_map.js _index): open addressing,
// FNV-1a over the key bytes (the Latin-1 character codes), linear probing,
// -1 = empty.  The same table the JS loop builds, without a per-character
// charCodeAt (C2: 1.96 M keys).
napi_value IndexKeys(napi_env env, napi_callback_info info) {
    size_t argc = 4;
    napi_value argv[4];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    bool isbuf = false;
    if (argc >= 4) napi_is_buffer(env, argv[0], &isbuf);
    napi_typedarray_type tt = napi_int8_array;
    size_t olen = 0;
    void *od = nullptr;
    if (!isbuf || napi_get_typedarray_info(env, argv[1], &tt, &olen, &od, nullptr, nullptr) != napi_ok ||
        tt != napi_float64_array) {
        napi_throw_type_error(env, nullptr, "indexKeys(keys Buffer, offsets Float64Array, n, cap)");
        return nullptr;
    }
    void *kd = nullptr;
    size_t klen = 0;
    NAPI_CALL(env, napi_get_buffer_info(env, argv[0], &kd, &klen));
    double n = 0, cap = 0;
    napi_get_value_double(env, argv[2], &n);
    napi_get_value_double(env, argv[3], &cap);
    const double *off = static_cast<const double *>(od);
    const uint64_t cn = (uint64_t)cap;
    if (n < 0 || (size_t)n + 1 > olen || cn == 0 || (cn & (cn - 1)) || cn < (uint64_t)n + 1 ||
        cn > 0x7FFFFFFFull || (n > 0 && off[(size_t)n] > (double)klen)) {
        napi_throw_range_error(env, nullptr, "indexKeys: bad sizes");
        return nullptr;
    }
    napi_value ab, ta;
    void *data = nullptr;
    NAPI_CALL(env, napi_create_arraybuffer(env, cn * 4, &data, &ab));
    int32_t *tab = static_cast<int32_t *>(data);
    memset(tab, 0xFF, cn * 4);
    const uint8_t *keys = static_cast<const uint8_t *>(kd);
    const uint32_t mask = (uint32_t)(cn - 1);
    // hashes first (a sequential pass), then the inserts with the home slots
    // prefetched a few keys ahead (the table is far larger than the caches)
    const size_t nn = (size_t)n;
    std::vector<uint32_t> hv(nn);
    for (size_t i = 0; i < nn; ++i) {
        uint32_t h = 0x811c9dc5u;
        for (uint64_t j = (uint64_t)off[i]; j < (uint64_t)off[i + 1]; ++j) h = (h ^ keys[j]) * 16777619u;
        hv[i] = h & mask;
    }
    constexpr size_t AHEAD = 16;
    for (size_t i = 0; i < nn; ++i) {
        if (i + AHEAD < nn) __builtin_prefetch(tab + hv[i + AHEAD], 1);
        uint32_t h = hv[i];
        while (tab[h] != -1) h = (h + 1) & mask;
        tab[h] = (int32_t)i;
    }
    NAPI_CALL(env, napi_create_typedarray(env, napi_int32_array, cn, ab, 0, &ta));
    return ta;
}

// KMERHIP_SEGV_TRACE=1 (diagnostics): a backtrace on stderr for a fatal signal
void segv_trace(int sig) {
    void *fr[64];
    const int n = backtrace(fr, 64);
    const char msg[] = "kmerhip: fatal signal, backtrace:\n";
    (void)!write(2, msg, sizeof(msg) - 1);
    backtrace_symbols_fd(fr, n, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}

napi_value Init(napi_env env, napi_value exports) {
    if (getenv("KMERHIP_SEGV_TRACE")) {
        signal(SIGSEGV, segv_trace);
        signal(SIGABRT, segv_trace);
    }
    napi_property_descriptor props[] = {
        {"open", nullptr, Open, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"countFile", nullptr, CountFile, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"countBuffer", nullptr, CountBuffer, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"close", nullptr, Close, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"version", nullptr, Version, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"dbOpen", nullptr, DbOpen, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"dbInfo", nullptr, DbInfo, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"dbClose", nullptr, DbClose, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"matchOpen", nullptr, MatchOpen, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"matchTemplates", nullptr, MatchTemplates, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"matchTemplateKmers", nullptr, MatchTemplateKmers, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"matchWinner", nullptr, MatchWinner, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"matchRemove", nullptr, MatchRemove, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"matchRemoved", nullptr, MatchRemoved, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"matchClose", nullptr, MatchClose, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
        {"indexKeys", nullptr, IndexKeys, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
    };
    napi_define_properties(env, exports, sizeof(props) / sizeof(props[0]), props);
    return exports;
}

}  // namespace

NAPI_MODULE(NODE_GYP_MODULE_NAME, Init)
