/*
 * talos_module.c — TEST INFRASTRUCTURE ONLY: a TaLoS TLS-processing module in
 * the shape of src/talos/enclaveshim/logpoint.c:127-135, linked into the
 * TaLoS-patched library in logpoint.o's place (Makefile.nosgx:633-634, "Add
 * files here for your TLS processing module").
 *
 * tls_processing_module_init() registers its callbacks through the reference
 * interface (tls_processing_interface.h:23-27).  The callbacks log every
 * plaintext chunk they are given — (SSL*, direction, length, FNV-1a 64 of the
 * bytes) — and count connections, so the loopback harness can check that the
 * module saw every application record at the patched call sites
 * (s3_pkt.c.patch:19-33 in do_ssl3_write, :39-52 in ssl3_read_bytes) and that
 * the bytes it saw are the plaintext.  With libtlsgpu.so preloaded, the
 * registration and the hook calls bind to libtlsgpu's implementation of the
 * interface (talos_amd/csrc/talos_hooks.cpp).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>

typedef struct ssl_st SSL;

void tls_processing_register_ssl_read_processing_cb(void (*cb)(const SSL *, char *, unsigned int *));
void tls_processing_register_ssl_write_processing_cb(void (*cb)(const SSL *, char *, unsigned int *));
void tls_processing_register_new_connection_cb(void (*cb)(const SSL *));
void tls_processing_register_free_connection_cb(void (*cb)(const SSL *));

struct talos_log_entry {
	const void *ssl;
	uint32_t dir;	/* 0 read (ssl3_read_bytes), 1 write (do_ssl3_write) */
	uint32_t len;
	uint64_t fnv;
};

#define LOG_CAP (1u << 20)
static struct talos_log_entry *entries;
static uint64_t n_entries, n_new, n_free;
static pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;

static uint64_t
fnv1a(const unsigned char *p, unsigned int n)
{
	uint64_t h = 0xcbf29ce484222325ull;
	for (unsigned int i = 0; i < n; i++)
		h = (h ^ p[i]) * 0x100000001b3ull;
	return h;
}

static void
log_chunk(const SSL *s, uint32_t dir, char *data, unsigned int *len)
{
	const uint64_t h = fnv1a((const unsigned char *)data, *len);
	pthread_mutex_lock(&mu);
	if (entries && n_entries < LOG_CAP)
		entries[n_entries++] = (struct talos_log_entry){s, dir, *len, h};
	pthread_mutex_unlock(&mu);
}

static void
on_read(const SSL *s, char *data, unsigned int *len)
{
	log_chunk(s, 0, data, len);
}

static void
on_write(const SSL *s, char *data, unsigned int *len)
{
	log_chunk(s, 1, data, len);
}

static void
on_new(const SSL *s)
{
	(void)s;
	pthread_mutex_lock(&mu);
	n_new++;
	pthread_mutex_unlock(&mu);
}

static void
on_free(const SSL *s)
{
	(void)s;
	pthread_mutex_lock(&mu);
	n_free++;
	pthread_mutex_unlock(&mu);
}

void
tls_processing_module_init(void)
{
	pthread_mutex_lock(&mu);
	if (!entries)
		entries = calloc(LOG_CAP, sizeof(*entries));
	pthread_mutex_unlock(&mu);
	tls_processing_register_ssl_read_processing_cb(on_read);
	tls_processing_register_ssl_write_processing_cb(on_write);
	tls_processing_register_new_connection_cb(on_new);
	tls_processing_register_free_connection_cb(on_free);
}

/* for the harness (dlsym): the log and the connection counts */
const struct talos_log_entry *
talos_module_log(uint64_t *n, uint64_t *new_conns, uint64_t *free_conns)
{
	pthread_mutex_lock(&mu);
	*n = n_entries;
	*new_conns = n_new;
	*free_conns = n_free;
	pthread_mutex_unlock(&mu);
	return entries;
}
