/*
 * tlsgpu_talos.h — TaLoS's TLS-processing interface as libtlsgpu.so exports it.
 *
 * Same names and signatures as the reference's
 * src/talos/enclaveshim/tls_processing_interface.h:23-49 (implementation:
 * tls_processing_interface.c:29-90), so a TaLoS module (e.g.
 * src/talos/enclaveshim/logpoint.c:127-135) registers its callbacks against the
 * engine unchanged, and a TaLoS-patched libssl (src/talos/patch/s3_pkt.c.patch,
 * ssl_lib.c.patch, bio_lib.c.patch) calls into it when libtlsgpu.so is
 * interposed.  Besides the patched record layer, the engine's host-delivery
 * paths fire the read / write callbacks (include/tlsgpu.h, "TaLoS
 * plaintext-processing hooks").
 *
 * One difference from the reference, on purpose: tls_processing_ssl_read /
 * _ssl_write also accept the BY-VALUE length the patched s3_pkt.c passes
 * (s3_pkt.c.patch:13-14 declares `unsigned int len`, the interface
 * `unsigned int *len`); the reference forwards that value as a pointer and a
 * module that reads *len faults.  How the third argument of these two entry
 * points is read is PROCESS-WIDE, chosen by the environment variable
 * TLSGPU_TALOS_LEN at load time (talos_amd/csrc/talos_hooks.cpp):
 *   "value"   always the by-value length (low 32 bits of the argument) — the
 *             setting for the TaLoS-patched record layer;
 *   "pointer" always a pointer, as declared;
 *   unset     a "pointer" below 64 KiB is taken as the length itself.  This
 *             relies on the caller zero-extending the 32-bit length into the
 *             64-bit argument register (gcc and clang do; the x86-64 SysV ABI
 *             leaves those bits undefined), so use "value" with a patched tree
 *             built by any other compiler.
 * The engine's own host paths always hand the callbacks real pointers.
 */
#ifndef TLSGPU_TALOS_H
#define TLSGPU_TALOS_H

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ssl_st SSL;

/* public: modules register their callbacks (tls_processing_interface.h:23-27) */
void tls_processing_register_ssl_read_processing_cb(void (*cb)(const SSL *, char *, unsigned int *));
void tls_processing_register_ssl_write_processing_cb(void (*cb)(const SSL *, char *, unsigned int *));
void tls_processing_register_set_ssl_type_cb(void (*cb)(const void *, const long));
void tls_processing_register_new_connection_cb(void (*cb)(const SSL *));
void tls_processing_register_free_connection_cb(void (*cb)(const SSL *));

/* private: called by TaLoS (tls_processing_interface.h:30-49) */
void ecall_tls_processing_module_init(void);	/* -> the module's tls_processing_module_init */
void tls_processing_ssl_read(const SSL *s, char *data, unsigned int *len);
void tls_processing_ssl_write(const SSL *s, char *data, unsigned int *len);
void tls_processing_set_ssl_type(const void *b, const long type);
void tls_processing_new_connection(const SSL *s);
void tls_processing_free_connection(const SSL *s);

#ifdef __cplusplus
}
#endif
#endif
