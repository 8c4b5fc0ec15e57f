// In-memory stand-in for the JVM side of JNI (TEST INFRASTRUCTURE ONLY; tests/test_jni_shim.py).
//
// The image has no JDK, so the shim spark-timeseries_amd/jni/sts_jni.cpp is
// linked here against:
//   * the JNIEnv / JavaVM members of tests/native/jni_stub/jni.h, implemented over a toy heap
//     (double[] and Object[] arrays, strings, classes, throwables; one pending exception);
//   * a CPU backend for the C-ABI functions the shim calls, built from the oracle's restated
//     primitives (oracle/sts_oracle.c) -- so what is checked is the SHIM: gathering a
//     partition's record arrays into one panel, scattering the results into a FRESH double[]
//     per record (each record owns its vector, S/TimeSeriesRDD.scala:538), length checks, and
//     the reference's exception classes.  The device path behind the same C ABI is checked by
//     the GPU tests.
// main() drives the *Records natives and the panel natives; prints "ok" on success.
#include <jni.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "sts.h"
extern "C" {
#include "sts_oracle.h"
}

// ---------------- the toy heap ----------------
namespace {

enum Kind { kDoubles = 1, kObjects, kString, kClass, kThrowable };
struct Obj {
    Kind kind;
    std::vector<double> d;
    std::vector<jobject> o;
    std::string s;   // string value / class name / throwable class
};
std::vector<std::unique_ptr<Obj>> g_heap;
std::unordered_map<const void*, Obj*> g_index;
Obj* g_pending = nullptr;   // the pending exception (a kThrowable)
int g_local_refs = 0, g_max_local_refs = 0;

template <class J>
J make(Kind k) {
    g_heap.emplace_back(new Obj{k, {}, {}, {}});
    Obj* o = g_heap.back().get();
    // the handle is the address of a one-byte marker owned by the object (the stub's _j* classes are empty)
    auto* h = new char;
    g_index[h] = o;
    if (++g_local_refs > g_max_local_refs) g_max_local_refs = g_local_refs;
    return reinterpret_cast<J>(h);
}
Obj* deref(const void* h) {
    auto it = g_index.find(h);
    return it == g_index.end() ? nullptr : it->second;
}
jdoubleArray new_doubles(const std::vector<double>& v) {
    jdoubleArray a = make<jdoubleArray>(kDoubles);
    deref(a)->d = v;
    return a;
}
jstring new_string(const char* s) {
    jstring a = make<jstring>(kString);
    deref(a)->s = s;
    return a;
}
void throw_named(const std::string& cls, const std::string& msg) {
    jthrowable t = make<jthrowable>(kThrowable);
    deref(t)->s = cls + ": " + msg;
    g_pending = deref(t);
}

}  // namespace

jclass JNIEnv::FindClass(const char* name) {
    jclass c = make<jclass>(kClass);
    deref(c)->s = name;
    return c;
}
jobject JNIEnv::NewGlobalRef(jobject obj) { return obj; }
void JNIEnv::DeleteLocalRef(jobject) { g_local_refs--; }
void JNIEnv::ExceptionClear() { g_pending = nullptr; }
jboolean JNIEnv::ExceptionCheck() { return g_pending != nullptr; }
jint JNIEnv::Throw(jthrowable obj) {
    g_pending = deref(obj);
    return 0;
}
jint JNIEnv::ThrowNew(jclass clazz, const char* msg) {
    throw_named(deref(clazz)->s, msg ? msg : "");
    return 0;
}
jmethodID JNIEnv::GetMethodID(jclass, const char*, const char*) { return reinterpret_cast<jmethodID>(1); }
jmethodID JNIEnv::GetStaticMethodID(jclass, const char*, const char*) { return reinterpret_cast<jmethodID>(1); }
jfieldID JNIEnv::GetStaticFieldID(jclass, const char*, const char*) { return reinterpret_cast<jfieldID>(1); }
jobject JNIEnv::GetStaticObjectField(jclass, jfieldID) { return new_string("NOT_ENOUGH_DATA_FOR_NUMBER_OF_PREDICTORS"); }
jobject JNIEnv::CallStaticObjectMethod(jclass, jmethodID, ...) { return new_string("boxed"); }
jobject JNIEnv::NewObject(jclass clazz, jmethodID, ...) {
    jthrowable t = make<jthrowable>(kThrowable);
    deref(t)->s = deref(clazz)->s + ": (constructed)";
    return t;
}
jobjectArray JNIEnv::NewObjectArray(jsize len, jclass, jobject init) {
    jobjectArray a = make<jobjectArray>(kObjects);
    deref(a)->o.assign((size_t)len, init);
    return a;
}
void JNIEnv::SetObjectArrayElement(jobjectArray array, jsize index, jobject val) {
    Obj* a = deref(array);
    if (index < 0 || (size_t)index >= a->o.size()) return throw_named("java/lang/ArrayIndexOutOfBoundsException", "set");
    a->o[(size_t)index] = val;
}
jobject JNIEnv::GetObjectArrayElement(jobjectArray array, jsize index) {
    Obj* a = deref(array);
    if (index < 0 || (size_t)index >= a->o.size()) {
        throw_named("java/lang/ArrayIndexOutOfBoundsException", "get");
        return nullptr;
    }
    if (a->o[(size_t)index]) g_local_refs++;
    return a->o[(size_t)index];
}
jdoubleArray JNIEnv::NewDoubleArray(jsize len) {
    jdoubleArray a = make<jdoubleArray>(kDoubles);
    deref(a)->d.assign((size_t)len, 0.0);
    return a;
}
jsize JNIEnv::GetArrayLength(jarray array) {
    Obj* a = deref(array);
    return (jsize)(a->kind == kDoubles ? a->d.size() : a->o.size());
}
void JNIEnv::GetDoubleArrayRegion(jdoubleArray array, jsize start, jsize len, jdouble* buf) {
    Obj* a = deref(array);
    if (start < 0 || len < 0 || (size_t)(start + len) > a->d.size())
        return throw_named("java/lang/ArrayIndexOutOfBoundsException", "region");
    std::memcpy(buf, a->d.data() + start, (size_t)len * sizeof(double));
}
void JNIEnv::SetDoubleArrayRegion(jdoubleArray array, jsize start, jsize len, const jdouble* buf) {
    Obj* a = deref(array);
    if (start < 0 || len < 0 || (size_t)(start + len) > a->d.size())
        return throw_named("java/lang/ArrayIndexOutOfBoundsException", "region");
    std::memcpy(a->d.data() + start, buf, (size_t)len * sizeof(double));
}
const char* JNIEnv::GetStringUTFChars(jstring str, jboolean*) { return deref(str)->s.c_str(); }
void JNIEnv::ReleaseStringUTFChars(jstring, const char*) {}
jboolean JNIEnv::IsSameObject(jobject a, jobject b) { return a == b; }
jint JavaVM::GetEnv(void** penv, jint) {
    static JNIEnv env;
    *penv = &env;
    return JNI_OK;
}

// ---------------- CPU backend of the C ABI calls the shim makes ----------------
namespace {
std::string g_err;
int fail(int st, const char* msg) {
    g_err = msg;
    return st;
}
}  // namespace

extern "C" {
const char* sts_last_error(void) { return g_err.c_str(); }
int sts_fill_method_from_name(const char* name) {
    if (!name) return -2;
    if (!std::strcmp(name, "linear")) return STS_FILL_LINEAR;
    if (!std::strcmp(name, "nearest")) return STS_FILL_NEAREST;
    if (!std::strcmp(name, "next")) return STS_FILL_NEXT;
    if (!std::strcmp(name, "previous")) return STS_FILL_PREVIOUS;
    if (!std::strcmp(name, "spline")) return STS_FILL_SPLINE;
    return -2;
}
int sts_host_alloc(size_t bytes, void** out) {
    // JNI_FAKE_NO_PIN=1: pinned memory cannot be had (the shim must fall back to the heap)
    const char* nopin = std::getenv("JNI_FAKE_NO_PIN");
    if (nopin && nopin[0] == '1') {
        *out = nullptr;
        return STS_ERR_HIP;
    }
    *out = std::malloc(bytes ? bytes : 16);
    return *out ? STS_OK : STS_ERR_HIP;
}
int sts_host_free(void* p) {
    std::free(p);
    return STS_OK;
}
int sts_fill_host(const double* in, double* out, int64_t S, int64_t T, int64_t ld, int method, int32_t* err) {
    for (int64_t s = 0; s < S; s++) {
        const int r = orc_fillts(in + s * ld, out + s * ld, T, method);   // ORC_* == STS_* codes
        if (err) err[s] = r;
        else if (r) return fail(r, r == STS_ERR_ALL_NAN ? "Input is all NaNs!" : "number of points");
    }
    return STS_OK;
}
int sts_fill_diff_ewma_host(const double* in, double* out, int64_t S, int64_t T, int64_t ld, int method, int lag,
                            const double* smoothing, int32_t*) {
    std::vector<double> f((size_t)T), d((size_t)T);
    for (int64_t s = 0; s < S; s++) {
        if (orc_fillts(in + s * ld, f.data(), T, method)) return fail(STS_ERR_ALL_NAN, "Input is all NaNs!");
        d = f;
        if (lag > 0 && orc_differences_at_lag(f.data(), d.data(), T, lag, lag)) return fail(STS_ERR_REQUIREMENT, "lag");
        orc_ewma_add(d.data(), out + s * ld, T, smoothing[s]);
    }
    return STS_OK;
}
int sts_ar_fit_remove_host(const double* in, double* out, int64_t S, int64_t T, int64_t ld, int p, int no_intercept,
                           double* c, double* coef, int32_t*) {
    if (T - p < p + 1) return fail(STS_ERR_NOT_ENOUGH_DATA, "not enough data");
    for (int64_t s = 0; s < S; s++) {
        if (orc_ar_fit(in + s * ld, T, p, no_intercept, c + s, coef + s * p)) return fail(STS_ERR_SINGULAR, "singular");
        orc_ar_remove(in + s * ld, out + s * ld, T, c[s], coef + s * p, p);
    }
    return STS_OK;
}
// the shim's other entry points are linked but not driven here
#define UNUSED_ENTRY(name, ...) \
    int name(__VA_ARGS__) { return fail(STS_ERR_NO_DEVICE, #name " is not part of the CPU stand-in"); }
UNUSED_ENTRY(sts_autocorr_host, const double*, int64_t, int64_t, int64_t, int, double*)
UNUSED_ENTRY(sts_fill_autocorr_host, const double*, double*, int64_t, int64_t, int64_t, int, int, double*, int32_t*)
UNUSED_ENTRY(sts_diff_at_lag_host, const double*, double*, int64_t, int64_t, int64_t, int, int)
UNUSED_ENTRY(sts_lag_matrix_host, const double*, double*, int64_t, int64_t, int64_t, int, int)
UNUSED_ENTRY(sts_ewma_add_host, const double*, double*, int64_t, int64_t, int64_t, const double*)
UNUSED_ENTRY(sts_ewma_remove_host, const double*, double*, int64_t, int64_t, int64_t, const double*)
UNUSED_ENTRY(sts_ewma_fit_host, const double*, int64_t, int64_t, int64_t, double*, int32_t*)
UNUSED_ENTRY(sts_garch_fit_host, const double*, int64_t, int64_t, int64_t, double*, int32_t*)
UNUSED_ENTRY(sts_argarch_fit_host, const double*, int64_t, int64_t, int64_t, double*, double*, double*, int32_t*)
UNUSED_ENTRY(sts_ar_fit_host, const double*, int64_t, int64_t, int64_t, int, int, double*, double*, int32_t*)
UNUSED_ENTRY(sts_ar_remove_host, const double*, double*, int64_t, int64_t, int64_t, const double*, const double*, int)
UNUSED_ENTRY(sts_ar_add_host, const double*, double*, int64_t, int64_t, int64_t, const double*, const double*, int)

// the shim's natives (sts_jni.cpp)
JNIEXPORT jint JNICALL JNI_OnLoad(JavaVM* vm, void*);
JNIEXPORT jobjectArray JNICALL Java_com_cloudera_sparkts_StsNative_fillRecords(JNIEnv*, jclass, jobjectArray, jlong,
                                                                               jstring);
JNIEXPORT jobjectArray JNICALL Java_com_cloudera_sparkts_StsNative_fillDiffEwmaRecords(JNIEnv*, jclass, jobjectArray,
                                                                                       jlong, jstring, jint,
                                                                                       jdoubleArray);
JNIEXPORT jobjectArray JNICALL Java_com_cloudera_sparkts_StsNative_arFitRemoveRecords(JNIEnv*, jclass, jobjectArray,
                                                                                      jlong, jint, jboolean,
                                                                                      jdoubleArray, jdoubleArray);
JNIEXPORT void JNICALL Java_com_cloudera_sparkts_StsNative_fill(JNIEnv*, jclass, jdoubleArray, jdoubleArray, jlong,
                                                                 jlong, jstring);
}  // extern "C"

// ---------------- the driver ----------------
namespace {
int g_fail = 0;
void check(bool ok, const char* what) {
    if (!ok) {
        std::printf("FAIL %s\n", what);
        g_fail++;
    }
}
bool same_bits(const double* a, const double* b, size_t n) {
    for (size_t i = 0; i < n; i++)
        if (std::memcmp(a + i, b + i, sizeof(double)) && !(std::isnan(a[i]) && std::isnan(b[i]))) return false;
    return true;
}
std::string pending_class() {
    if (!g_pending) return "";
    const std::string& s = g_pending->s;
    return s.substr(0, s.find(':'));
}
}  // namespace

int main() {
    JavaVM vm;
    check(JNI_OnLoad(&vm, nullptr) == JNI_VERSION_1_6, "JNI_OnLoad");
    JNIEnv* env = nullptr;
    vm.GetEnv(reinterpret_cast<void**>(&env), JNI_VERSION_1_6);
    const int S = 6, T = 40;
    // a partition of S records, each its own double[] (with NaN gaps)
    std::vector<std::vector<double>> data(S, std::vector<double>(T));
    for (int s = 0; s < S; s++)
        for (int t = 0; t < T; t++) data[s][t] = ((t * 7 + s * 3) % 11 == 4 && t > 0 && t < T - 1) ? NAN : 100.0 + s + 0.37 * t * ((t + s) % 3);
    jobjectArray recs = env->NewObjectArray(S, env->FindClass("[D"), nullptr);
    std::vector<jdoubleArray> in_arrays;
    for (int s = 0; s < S; s++) {
        in_arrays.push_back(new_doubles(data[s]));
        env->SetObjectArrayElement(recs, s, in_arrays.back());
    }
    jclass cls = env->FindClass("com/cloudera/sparkts/StsNative");

    // ---- fillRecords: fresh, distinct arrays per record, oracle values, inputs untouched ----
    for (const char* m : {"linear", "previous", "next", "nearest", "spline"}) {
        jobjectArray out = Java_com_cloudera_sparkts_StsNative_fillRecords(env, cls, recs, T, new_string(m));
        check(out && !g_pending, m);
        if (!out) continue;
        check(env->GetArrayLength(out) == S, "record count");
        std::vector<const void*> seen;
        for (int s = 0; s < S; s++) {
            jobject r = deref(out)->o[(size_t)s];
            check(r != nullptr && deref(r)->kind == kDoubles && deref(r)->d.size() == (size_t)T, "record array");
            for (const void* q : seen) check(q != r, "records share an array");
            for (jdoubleArray a : in_arrays) check(r != a, "output aliases an input record");
            seen.push_back(r);
            std::vector<double> want((size_t)T);
            orc_fillts(data[s].data(), want.data(), T, sts_fill_method_from_name(m));
            check(same_bits(deref(r)->d.data(), want.data(), (size_t)T), "fill values");
            check(same_bits(deref(in_arrays[(size_t)s])->d.data(), data[s].data(), (size_t)T), "input untouched");
        }
    }
    // ---- errors: the reference's exception classes ----
    env->ExceptionClear();
    check(!Java_com_cloudera_sparkts_StsNative_fillRecords(env, cls, recs, T, new_string("cubic")) &&
              pending_class() == "java/lang/UnsupportedOperationException",
          "unknown method -> UnsupportedOperationException");
    env->ExceptionClear();
    {
        // "spline" stays a working method (S/UnivariateTimeSeries.scala:147): fresh records, the
        // restated commons-math3 spline's bits; a record with fewer than 3 points throws
        // commons-math3 NumberIsTooSmallException, as SplineInterpolator.interpolate does
        jobjectArray got = Java_com_cloudera_sparkts_StsNative_fillRecords(env, cls, recs, T, new_string("spline"));
        check(got && !env->ExceptionCheck(), "spline -> filled records");
        for (int64_t s = 0; got && s < S; s++) {
            std::vector<double> want((size_t)T);
            check(orc_fill_spline(data[s].data(), want.data(), T) == 0, "spline oracle");
            jdoubleArray r = static_cast<jdoubleArray>(env->GetObjectArrayElement(got, (jsize)s));
            check(same_bits(deref(r)->d.data(), want.data(), (size_t)T), "spline values");
        }
        env->ExceptionClear();
        jobjectArray few = env->NewObjectArray(2, env->FindClass("[D"), nullptr);
        std::vector<double> two((size_t)T, NAN);
        two[1] = 1.0;
        two[3] = 2.0;
        env->SetObjectArrayElement(few, 0, new_doubles(data[0]));
        env->SetObjectArrayElement(few, 1, new_doubles(two));
        check(!Java_com_cloudera_sparkts_StsNative_fillRecords(env, cls, few, T, new_string("spline")) &&
                  pending_class() == "org/apache/commons/math3/exception/NumberIsTooSmallException",
              "spline on 2 points -> NumberIsTooSmallException");
        env->ExceptionClear();
    }
    jobjectArray ragged = env->NewObjectArray(2, env->FindClass("[D"), nullptr);
    env->SetObjectArrayElement(ragged, 0, new_doubles(data[0]));
    env->SetObjectArrayElement(ragged, 1, new_doubles(std::vector<double>(T - 1, 1.0)));
    check(!Java_com_cloudera_sparkts_StsNative_fillRecords(env, cls, ragged, T, new_string("linear")) &&
              pending_class() == "java/lang/IllegalArgumentException",
          "ragged records -> IllegalArgumentException");
    env->ExceptionClear();
    jobjectArray allnan = env->NewObjectArray(1, env->FindClass("[D"), nullptr);
    env->SetObjectArrayElement(allnan, 0, new_doubles(std::vector<double>{5.0, NAN}));   // [5, NaN]: throws
    check(!Java_com_cloudera_sparkts_StsNative_fillRecords(env, cls, allnan, 2, new_string("nearest")) &&
              g_pending && g_pending->s == "java/lang/IllegalArgumentException: Input is all NaNs!",
          "nearest [5, NaN] -> IllegalArgumentException(Input is all NaNs!)");
    env->ExceptionClear();
    jobjectArray empty = env->NewObjectArray(0, env->FindClass("[D"), nullptr);
    jobjectArray eo = Java_com_cloudera_sparkts_StsNative_fillRecords(env, cls, empty, T, new_string("linear"));
    check(eo && env->GetArrayLength(eo) == 0 && !g_pending, "empty partition");

    // ---- fillDiffEwmaRecords / arFitRemoveRecords ----
    std::vector<double> sm(S);
    for (int s = 0; s < S; s++) sm[(size_t)s] = 0.1 + 0.1 * s;
    jobjectArray o2 = Java_com_cloudera_sparkts_StsNative_fillDiffEwmaRecords(env, cls, recs, T, new_string("previous"), 1,
                                                                               new_doubles(sm));
    check(o2 && !g_pending, "fillDiffEwmaRecords");
    for (int s = 0; o2 && s < S; s++) {
        std::vector<double> f((size_t)T), d((size_t)T), want((size_t)T);
        orc_fill_previous(data[s].data(), f.data(), T);
        d = f;
        orc_differences_at_lag(f.data(), d.data(), T, 1, 1);
        orc_ewma_add(d.data(), want.data(), T, sm[(size_t)s]);
        check(same_bits(deref(deref(o2)->o[(size_t)s])->d.data(), want.data(), (size_t)T), "fill-diff-ewma values");
    }
    check(!Java_com_cloudera_sparkts_StsNative_fillDiffEwmaRecords(env, cls, recs, T, new_string("previous"), 1,
                                                                   new_doubles(std::vector<double>(S - 1, 0.2))) &&
              pending_class() == "java/lang/IllegalArgumentException",
          "short smoothing array");
    env->ExceptionClear();
    const int p = 2;
    jobjectArray filled = Java_com_cloudera_sparkts_StsNative_fillRecords(env, cls, recs, T, new_string("linear"));
    jdoubleArray jc = new_doubles(std::vector<double>(S)), jk = new_doubles(std::vector<double>(S * p));
    jobjectArray o3 = Java_com_cloudera_sparkts_StsNative_arFitRemoveRecords(env, cls, filled, T, p, 0, jc, jk);
    check(o3 && !g_pending, "arFitRemoveRecords");
    for (int s = 0; o3 && s < S; s++) {
        const std::vector<double>& x = deref(deref(filled)->o[(size_t)s])->d;
        double c = 0, k[2];
        orc_ar_fit(x.data(), T, p, 0, &c, k);
        std::vector<double> want((size_t)T);
        orc_ar_remove(x.data(), want.data(), T, c, k, p);
        check(same_bits(deref(deref(o3)->o[(size_t)s])->d.data(), want.data(), (size_t)T), "AR residual values");
        check(same_bits(&deref(jc)->d[(size_t)s], &c, 1) && same_bits(&deref(jk)->d[(size_t)s * p], k, 2), "AR model");
    }
    check(!Java_com_cloudera_sparkts_StsNative_arFitRemoveRecords(env, cls, filled, 4, p, 0, jc, jk) &&
              pending_class() == "java/lang/IllegalArgumentException",
          "records longer than T -> IllegalArgumentException");
    env->ExceptionClear();

    // ---- an oversized partition: no pinned or heap buffer can be had -> OutOfMemoryError, not an
    //      abort (std::bad_alloc must not leave a JNIEXPORT function) ----
    const jlong huge = jlong(1) << 40;   // 8 TB of doubles for one record
    check(!Java_com_cloudera_sparkts_StsNative_fillRecords(env, cls, recs, huge, new_string("linear")) &&
              pending_class() == "java/lang/OutOfMemoryError",
          "oversized partition -> OutOfMemoryError");
    env->ExceptionClear();
    check(!Java_com_cloudera_sparkts_StsNative_arFitRemoveRecords(env, cls, recs, huge, 2, 0, jc, jk) &&
              pending_class() == "java/lang/OutOfMemoryError",
          "oversized AR partition -> OutOfMemoryError");
    env->ExceptionClear();

    // ---- the panel form still works (one shared array in, one out) ----
    std::vector<double> flat;
    for (int s = 0; s < S; s++) flat.insert(flat.end(), data[s].begin(), data[s].end());
    jdoubleArray pin = new_doubles(flat), pout = new_doubles(std::vector<double>(flat.size()));
    Java_com_cloudera_sparkts_StsNative_fill(env, cls, pin, pout, S, T, new_string("linear"));
    check(!g_pending, "panel fill");
    for (int s = 0; s < S; s++) {
        std::vector<double> want((size_t)T);
        orc_fill_linear(data[s].data(), want.data(), T);
        check(same_bits(deref(pout)->d.data() + (size_t)s * T, want.data(), (size_t)T), "panel fill values");
    }
    if (g_fail) return 1;
    std::puts("ok");
    return 0;
}
