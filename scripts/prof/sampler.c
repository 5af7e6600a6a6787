// sampler.c -- a tiny in-process PC sampler for host-side profiling (dev tool; no perf in the image).
// Loaded with ctypes (never preloaded): sampler_start(usec) arms a CLOCK_MONOTONIC timer that raises
// SIGPROF; the handler records the interrupted PC while sampler_phase(tag > 0) is set.  sampler_stop
// writes "tag pc object base symbol" lines (dladdr) for scripts/prof/report.py to attribute.
// build: gcc -O2 -fPIC -shared -o /tmp/libfc2_sampler.so scripts/prof/sampler.c -lrt -ldl
#define _GNU_SOURCE
#include <dlfcn.h>
#include <execinfo.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <time.h>
#include <ucontext.h>
#include <stdlib.h>
#include <sys/syscall.h>
#include <sys/time.h>
#include <unistd.h>

#define MAXS (1 << 20)
#define DEPTH 12
static uintptr_t ips[MAXS];
static void *stk[MAXS][DEPTH];
static unsigned char nstk[MAXS];
static unsigned char tags[MAXS];
static volatile int n_samples;
static volatile int cur_tag;
static timer_t tid;

static void on_prof(int sig, siginfo_t *si, void *ucv) {
    (void)sig; (void)si;
    const int t = cur_tag;
    if (t <= 0) return;
    const ucontext_t *uc = (const ucontext_t *)ucv;
    const int i = __sync_fetch_and_add(&n_samples, 1);
    if (i < MAXS) {
        ips[i] = (uintptr_t)uc->uc_mcontext.gregs[REG_RIP];
        tags[i] = (unsigned char)t;
        nstk[i] = (unsigned char)backtrace(stk[i], DEPTH);   // handler, trampoline, then the interrupted frames
    }
}

/* FC2_SAMPLE_ALL: a CLOCK_MONOTONIC timer per thread (hrtimer resolution, unlike the tick-driven CPU
   clocks), each signalling its own thread; a monitor thread arms one for every new thread found in
   /proc/self/task.  Samples of blocked threads land in the blocking call (report.py --drop-waits). */
#include <dirent.h>
#include <pthread.h>
#define MAXT 512
static int n_armed;
static pid_t armed[MAXT];
static timer_t armed_timer[MAXT];
static volatile int monitor_stop;
static pthread_t monitor;
static int sample_usec;

static int arm(pid_t t) {
    for (int i = 0; i < n_armed; ++i)
        if (armed[i] == t) return 0;
    if (n_armed >= MAXT) return -1;
    struct sigevent ev;
    memset(&ev, 0, sizeof ev);
    ev.sigev_signo = SIGPROF;
    ev.sigev_notify = SIGEV_THREAD_ID;
    ev._sigev_un._tid = t;
    timer_t tm;
    if (timer_create(CLOCK_MONOTONIC, &ev, &tm)) return -1;
    struct itimerspec it;
    it.it_interval.tv_sec = 0;
    it.it_interval.tv_nsec = (long)sample_usec * 1000L;
    it.it_value = it.it_interval;
    timer_settime(tm, 0, &it, 0);
    armed[n_armed] = t;
    armed_timer[n_armed++] = tm;
    return 1;
}

static void *monitor_loop(void *arg) {
    (void)arg;
    const pid_t self = (pid_t)syscall(SYS_gettid);
    while (!monitor_stop) {
        DIR *d = opendir("/proc/self/task");
        if (d) {
            struct dirent *e;
            while ((e = readdir(d)))
                if (e->d_name[0] != '.') {
                    const pid_t t = (pid_t)atoi(e->d_name);
                    if (t != self) arm(t);
                }
            closedir(d);
        }
        usleep(2000);
    }
    return 0;
}

int sampler_start(int usec) {
    void *warm[4];
    backtrace(warm, 4);                          // loads the unwinder outside the signal handler
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = on_prof;
    sa.sa_flags = SA_SIGINFO | SA_RESTART;
    if (sigaction(SIGPROF, &sa, 0)) return -1;
    struct sigevent ev;
    memset(&ev, 0, sizeof ev);
    ev.sigev_signo = SIGPROF;
    if (getenv("FC2_SAMPLE_ALL")) {
        sample_usec = usec;
        monitor_stop = 0;
        return pthread_create(&monitor, 0, monitor_loop, 0);
    }
    if (getenv("FC2_SAMPLE_PROCESS")) {          /* every thread, on the process's CPU clock (ITIMER_PROF:
                                                    the signal goes to the thread that used the CPU) */
        struct itimerval iv;
        iv.it_interval.tv_sec = 0;
        iv.it_interval.tv_usec = usec;
        iv.it_value = iv.it_interval;
        tid = 0;
        return setitimer(ITIMER_PROF, &iv, 0);
    }
    if (getenv("FC2_SAMPLE_THREAD")) {           /* only the calling thread, on its own CPU clock */
        ev.sigev_notify = SIGEV_THREAD_ID;
        ev._sigev_un._tid = (pid_t)syscall(SYS_gettid);
        if (timer_create(CLOCK_THREAD_CPUTIME_ID, &ev, &tid)) return -2;
    } else {
        ev.sigev_notify = SIGEV_SIGNAL;
        if (timer_create(CLOCK_MONOTONIC, &ev, &tid)) return -2;
    }
    struct itimerspec it;
    it.it_interval.tv_sec = 0;
    it.it_interval.tv_nsec = (long)usec * 1000L;
    it.it_value = it.it_interval;
    return timer_settime(tid, 0, &it, 0);
}

void sampler_phase(int tag) { cur_tag = tag; }

int sampler_stop(const char *path) {
    cur_tag = 0;
    if (getenv("FC2_SAMPLE_ALL")) {
        monitor_stop = 1;
        pthread_join(monitor, 0);
        for (int i = 0; i < n_armed; ++i) timer_delete(armed_timer[i]);
        n_armed = 0;
    } else
    if (getenv("FC2_SAMPLE_PROCESS")) {
        struct itimerval iv;
        memset(&iv, 0, sizeof iv);
        setitimer(ITIMER_PROF, &iv, 0);
    } else {
        timer_delete(tid);
    }
    FILE *f = fopen(path, "w");
    if (!f) return -1;
    const int n = n_samples < MAXS ? n_samples : MAXS;
    for (int i = 0; i < n; ++i) {
        Dl_info d;
        memset(&d, 0, sizeof d);
        dladdr((void *)ips[i], &d);
        fprintf(f, "%d %lx %s %lx %s", tags[i], (unsigned long)ips[i], d.dli_fname ? d.dli_fname : "?",
                (unsigned long)(uintptr_t)d.dli_fbase, d.dli_sname ? d.dli_sname : "?");
        // the callers: frames after the interrupted PC, as object+offset
        int k = 0;
        while (k < nstk[i] && (uintptr_t)stk[i][k] != ips[i]) ++k;
        for (++k; k < nstk[i]; ++k) {
            Dl_info c;
            memset(&c, 0, sizeof c);
            dladdr(stk[i][k], &c);
            fprintf(f, " %s+%lx", c.dli_fname ? c.dli_fname : "?",
                    (unsigned long)((uintptr_t)stk[i][k] - (uintptr_t)c.dli_fbase));
        }
        fputc('\n', f);
    }
    fclose(f);
    return n;
}
