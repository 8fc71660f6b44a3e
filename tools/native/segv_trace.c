/* Diagnosis only: on SIGSEGV print the native backtrace (execinfo) and the faulting address to stderr, then hand
 * the signal to the handler that was installed before (Python's faulthandler, which prints the Python stacks).
 * Loaded with ctypes by tools/diag_capacity_capture.py; build: tools/native/build_segv_trace.sh. */
#define _GNU_SOURCE
#include <execinfo.h>
#include <signal.h>
#include <stdio.h>
#include <string.h>
#include <unistd.h>

static struct sigaction g_old;

static void on_segv(int sig, siginfo_t* si, void* uc) {
    void* bt[96];
    char msg[96];
    int n = backtrace(bt, 96);
    int len = snprintf(msg, sizeof msg, "segv_trace: signal %d at address %p, %d frames\n", sig, si->si_addr, n);
    if (len > 0) write(2, msg, (size_t)len);
    backtrace_symbols_fd(bt, n, 2);
    sigaction(SIGSEGV, &g_old, NULL);
    if (g_old.sa_flags & SA_SIGINFO) {
        if (g_old.sa_sigaction) g_old.sa_sigaction(sig, si, uc);
    } else if (g_old.sa_handler != SIG_DFL && g_old.sa_handler != SIG_IGN) {
        g_old.sa_handler(sig);
    }
    raise(sig);
}

int segv_trace_install(void) {
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = on_segv;
    sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
    sigemptyset(&sa.sa_mask);
    return sigaction(SIGSEGV, &sa, &g_old);
}
