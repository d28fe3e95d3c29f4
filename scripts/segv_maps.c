/* Diagnostic (profiling runs only): on SIGSEGV write the faulting address, the PC, the faulting
 * thread's kernel tid and name, and /proc/self/maps to a file, then hand the signal to the handler
 * that was installed before (the profiler's).  mz_segv_maps_snapshot writes the same maps at any
 * time (a run that completes).  Loaded by bench.py through ctypes when MZ_SEGV_MAPS=<file>.
 * Build: gcc -O2 -shared -fPIC scripts/segv_maps.c -o scripts/_segv_maps.so */
#define _GNU_SOURCE
#include <fcntl.h>
#include <signal.h>
#include <string.h>
#include <sys/syscall.h>
#include <ucontext.h>
#include <unistd.h>
#include <pthread.h>

static struct sigaction prev;
static char out_path[1024];

static void put(int fd, const char *s) { (void)!write(fd, s, strlen(s)); }
static void hex(int fd, unsigned long v) {
    char b[20];
    b[0] = '0';
    b[1] = 'x';
    for (int i = 0; i < 16; ++i) {
        int d = (int)((v >> (60 - 4 * i)) & 15);
        b[2 + i] = (char)(d < 10 ? '0' + d : 'a' + d - 10);
    }
    b[18] = '\n';
    (void)!write(fd, b, 19);
}
static void dec(int fd, long v) {
    char b[24];
    int n = 0;
    if (v == 0) b[n++] = '0';
    while (v > 0 && n < 22) {
        b[n++] = (char)('0' + v % 10);
        v /= 10;
    }
    for (int i = n - 1; i >= 0; --i) (void)!write(fd, &b[i], 1);
    (void)!write(fd, "\n", 1);
}
static void copy_file(int fd, const char *src) {
    int m = open(src, O_RDONLY);
    if (m < 0) return;
    char buf[4096];
    ssize_t n;
    while ((n = read(m, buf, sizeof buf)) > 0) (void)!write(fd, buf, (size_t)n);
    close(m);
}

static void handler(int sig, siginfo_t *si, void *ucv) {
    int fd = open(out_path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (fd >= 0) {
        ucontext_t *uc = (ucontext_t *)ucv;
        put(fd, "signal ");
        dec(fd, sig);
        put(fd, "fault_addr ");
        hex(fd, (unsigned long)si->si_addr);
        put(fd, "pc ");
        hex(fd, (unsigned long)uc->uc_mcontext.gregs[REG_RIP]);
        const long tid = syscall(SYS_gettid);
        put(fd, "tid ");
        dec(fd, tid);
        put(fd, "pthread_self ");
        hex(fd, (unsigned long)pthread_self());
        char comm[64] = "/proc/self/task/";
        char num[24];
        int n = 0;
        long v = tid;
        do {
            num[n++] = (char)('0' + v % 10);
            v /= 10;
        } while (v > 0);
        int k = (int)strlen(comm);
        for (int i = n - 1; i >= 0; --i) comm[k++] = num[i];
        strcpy(comm + k, "/comm");
        put(fd, "thread_name ");
        copy_file(fd, comm);
        put(fd, "--- /proc/self/maps ---\n");
        copy_file(fd, "/proc/self/maps");
        close(fd);
    }
    sigaction(SIGSEGV, &prev, 0);  /* the previous handler gets the re-raised fault */
}

int mz_segv_maps_install(const char *path) {
    strncpy(out_path, path, sizeof out_path - 1);
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = handler;
    sa.sa_flags = SA_SIGINFO;
    sigemptyset(&sa.sa_mask);
    return sigaction(SIGSEGV, &sa, &prev);
}

int mz_segv_maps_snapshot(const char *path) {
    int fd = open(path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (fd < 0) return -1;
    copy_file(fd, "/proc/self/maps");
    close(fd);
    return 0;
}
