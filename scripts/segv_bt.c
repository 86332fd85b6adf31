// Native backtrace on SIGSEGV / SIGABRT for a Python process (scripts/graph_capture_repro.py): install() chains in
// front of the handler already installed (Python's faulthandler), prints the native frames with backtrace_symbols_fd
// to stderr, then hands over to the previous handler. Host-side only.
//   gcc -O1 -g -shared -fPIC scripts/segv_bt.c -o scripts/bin/libsegv_bt.so
#define _GNU_SOURCE
#include <execinfo.h>
#include <signal.h>
#include <string.h>
#include <unistd.h>

static struct sigaction prev_segv, prev_abrt;

static void handler(int sig, siginfo_t* info, void* uc) {
    void* frames[64];
    const char msg[] = "\n[segv_bt] native backtrace:\n";
    write(2, msg, sizeof(msg) - 1);
    int n = backtrace(frames, 64);
    backtrace_symbols_fd(frames, n, 2);
    struct sigaction* p = sig == SIGSEGV ? &prev_segv : &prev_abrt;
    sigaction(sig, p, NULL);
    if (p->sa_flags & SA_SIGINFO) {
        if (p->sa_sigaction) p->sa_sigaction(sig, info, uc);
    } else if (p->sa_handler != SIG_DFL && p->sa_handler != SIG_IGN) {
        p->sa_handler(sig);
    }
    raise(sig);
}

int install(void) {
    struct sigaction sa;
    memset(&sa, 0, sizeof(sa));
    sa.sa_sigaction = handler;
    sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
    sigemptyset(&sa.sa_mask);
    if (sigaction(SIGSEGV, &sa, &prev_segv)) return -1;
    if (sigaction(SIGABRT, &sa, &prev_abrt)) return -1;
    return 0;
}
