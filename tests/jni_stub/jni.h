/* Test-only: the subset of the JNI declarations (JNI spec, "JNI Types and
 * Data Structures" / "JNI Functions") that integration/jni/capf_jni.cpp uses,
 * so tests/test_jni_shim.py can type-check the shim with g++ -fsyntax-only in
 * this JDK-less image.  Not used to build anything; a real build compiles
 * against $JAVA_HOME/include/jni.h. */
#ifndef CAPF_TEST_JNI_STUB_H
#define CAPF_TEST_JNI_STUB_H
#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL

typedef int8_t jbyte;
typedef int32_t jint;
typedef int64_t jlong;
typedef uint8_t jboolean;
typedef double jdouble;
typedef jint jsize;

class _jobject {};
class _jclass : public _jobject {};
class _jstring : public _jobject {};
class _jthrowable : public _jobject {};
class _jarray : public _jobject {};
class _jobjectArray : public _jarray {};
class _jintArray : public _jarray {};
class _jlongArray : public _jarray {};
class _jdoubleArray : public _jarray {};
class _jbooleanArray : public _jarray {};
class _jbyteArray : public _jarray {};
typedef _jobject *jobject;
typedef _jclass *jclass;
typedef _jstring *jstring;
typedef _jthrowable *jthrowable;
typedef _jarray *jarray;
typedef _jobjectArray *jobjectArray;
typedef _jintArray *jintArray;
typedef _jlongArray *jlongArray;
typedef _jdoubleArray *jdoubleArray;
typedef _jbooleanArray *jbooleanArray;
typedef _jbyteArray *jbyteArray;
struct _jmethodID;
struct _jfieldID;
typedef _jmethodID *jmethodID;
typedef _jfieldID *jfieldID;

struct JNIEnv {
  jclass FindClass(const char *name);
  jclass GetObjectClass(jobject obj);
  jmethodID GetMethodID(jclass clazz, const char *name, const char *sig);
  jfieldID GetFieldID(jclass clazz, const char *name, const char *sig);
  jobject GetObjectField(jobject obj, jfieldID field);
  jobject NewObject(jclass clazz, jmethodID ctor, ...);
  jint Throw(jthrowable obj);
  jint ThrowNew(jclass clazz, const char *message);
  jstring NewStringUTF(const char *utf);
  const char *GetStringUTFChars(jstring str, jboolean *is_copy);
  void ReleaseStringUTFChars(jstring str, const char *chars);
  jsize GetArrayLength(jarray array);
  jobjectArray NewObjectArray(jsize len, jclass clazz, jobject init);
  jobject GetObjectArrayElement(jobjectArray array, jsize index);
  void SetObjectArrayElement(jobjectArray array, jsize index, jobject val);
  void GetIntArrayRegion(jintArray array, jsize start, jsize len, jint *buf);
  void GetLongArrayRegion(jlongArray array, jsize start, jsize len, jlong *buf);
  void GetDoubleArrayRegion(jdoubleArray array, jsize start, jsize len, jdouble *buf);
  void GetBooleanArrayRegion(jbooleanArray array, jsize start, jsize len, jboolean *buf);
  void SetLongArrayRegion(jlongArray array, jsize start, jsize len, const jlong *buf);
  void SetDoubleArrayRegion(jdoubleArray array, jsize start, jsize len, const jdouble *buf);
  jbyteArray NewByteArray(jsize len);
  void GetByteArrayRegion(jbyteArray array, jsize start, jsize len, jbyte *buf);
  void SetByteArrayRegion(jbyteArray array, jsize start, jsize len, const jbyte *buf);
  void *GetDirectBufferAddress(jobject buf);
  jlong GetDirectBufferCapacity(jobject buf);
  void DeleteLocalRef(jobject obj);
};

#endif
