/* Minimal STAND-IN for the JNI C++ interface -- only the types and JNIEnv / JavaVM members
 * spark-timeseries_amd/jni/sts_jni.cpp uses, with the JDK's signatures, so that
 * tests/test_jni_shim.py can type-check the shim in an image without a JDK, and link it
 * against tests/native/jni_fake_env.cpp (an in-memory stand-in JVM heap that implements these
 * members) to exercise the shim's gather / scatter and exception paths on the CPU.  The
 * product shim is built against a real JDK's jni.h (Makefile target `jni`). */
#pragma once
#include <cstdarg>
#include <cstdint>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_OK 0
#define JNI_FALSE 0
#define JNI_TRUE 1
#define JNI_ERR (-1)
#define JNI_VERSION_1_6 0x00010006

typedef int32_t jint;
typedef int64_t jlong;
typedef uint8_t jboolean;
typedef double jdouble;
typedef jint jsize;

class _jobject {};
class _jclass : public _jobject {};
class _jthrowable : public _jobject {};
class _jstring : public _jobject {};
class _jarray : public _jobject {};
class _jdoubleArray : public _jarray {};
class _jobjectArray : public _jarray {};
typedef _jobject* jobject;
typedef _jclass* jclass;
typedef _jthrowable* jthrowable;
typedef _jstring* jstring;
typedef _jarray* jarray;
typedef _jdoubleArray* jdoubleArray;
typedef _jobjectArray* jobjectArray;
struct _jmethodID;
typedef _jmethodID* jmethodID;
struct _jfieldID;
typedef _jfieldID* jfieldID;

struct JNIEnv {
    jclass FindClass(const char* name);
    jobject NewGlobalRef(jobject obj);
    void DeleteLocalRef(jobject obj);
    void ExceptionClear();
    jboolean ExceptionCheck();
    jint Throw(jthrowable obj);
    jint ThrowNew(jclass clazz, const char* msg);
    jmethodID GetMethodID(jclass clazz, const char* name, const char* sig);
    jmethodID GetStaticMethodID(jclass clazz, const char* name, const char* sig);
    jfieldID GetStaticFieldID(jclass clazz, const char* name, const char* sig);
    jobject GetStaticObjectField(jclass clazz, jfieldID fieldID);
    jobject CallStaticObjectMethod(jclass clazz, jmethodID methodID, ...);
    jobject NewObject(jclass clazz, jmethodID methodID, ...);
    jobjectArray NewObjectArray(jsize len, jclass clazz, jobject init);
    void SetObjectArrayElement(jobjectArray array, jsize index, jobject val);
    jobject GetObjectArrayElement(jobjectArray array, jsize index);
    jdoubleArray NewDoubleArray(jsize len);
    jsize GetArrayLength(jarray array);
    void GetDoubleArrayRegion(jdoubleArray array, jsize start, jsize len, jdouble* buf);
    void SetDoubleArrayRegion(jdoubleArray array, jsize start, jsize len, const jdouble* buf);
    const char* GetStringUTFChars(jstring str, jboolean* isCopy);
    void ReleaseStringUTFChars(jstring str, const char* chars);
    jboolean IsSameObject(jobject obj1, jobject obj2);
};

struct JavaVM {
    jint GetEnv(void** penv, jint version);
};
