package jepsen.etcdemo;

import com.sun.jna.Native;
import com.sun.jna.Pointer;

/**
 * JNA direct mapping of liblincheck.so (include/lincheck.h): each static
 * native method is bound to the C symbol of the same name when the class
 * loads (Native.register), so a call costs a JNI transition, not a
 * reflective Function.invoke.  JNA 4.1.0 is already on the demo's classpath
 * (jepsen.etcdemo.iml:61-62); add this file to the project's
 * :java-source-paths.  Out-parameters (lc_ctx **, lc_packed **) are passed
 * as 8-byte Memory blocks; arrays of keys and report words as long[].
 *
 * NOT COMPILED IN THIS REPOSITORY: the build container has no JDK.
 */
public final class LincheckNative {
    static {
        Native.register("lincheck");
    }

    private LincheckNative() {}

    public static native int lc_abi_version();
    public static native String lc_last_error();
    public static native int lc_device_count();

    public static native int lc_create(Pointer opts, Pointer outCtx);
    public static native void lc_destroy(Pointer ctx);

    public static native int lc_pack(Pointer history, Pointer packOpts, Pointer outPacked);
    public static native void lc_packed_free(Pointer packed);
    public static native int lc_packed_view(Pointer packed, Pointer batch);
    public static native int lc_packed_keys(Pointer packed, long[] out);
    public static native String lc_packed_key_error(Pointer packed, long i);
    public static native long lc_packed_state_map(Pointer packed, long i, int s, long[] regs, long[] vals, long cap);

    public static native int lc_check_batch(Pointer ctx, Pointer batch, Pointer result, Pointer stats);

    public static native long lc_report(Pointer packed, long i, int valid, int failEvent, Pointer finalConfigs,
                                        int nFinal, int maxPaths, long[] out, long cap);
    public static native long lc_report_wgl(Pointer packed, long i, int valid, int failEvent, Pointer finalConfigs,
                                            int nFinal, int maxPaths, long[] out, long cap);
}
