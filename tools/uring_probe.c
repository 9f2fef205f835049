/* Is io_uring available to this process (a seccomp profile may refuse
 * io_uring_setup)?  One JSON line.  Build: gcc -O2 -o tools/_abx/uring_probe tools/uring_probe.c */
#include <errno.h>
#include <linux/io_uring.h>
#include <stdio.h>
#include <string.h>
#include <sys/syscall.h>
#include <unistd.h>
int main(void) {
    struct io_uring_params p;
    memset(&p, 0, sizeof p);
    long fd = syscall(__NR_io_uring_setup, 8, &p);
    if (fd < 0) { printf("{\"io_uring_setup\": \"refused\", \"errno\": %d, \"error\": \"%s\"}\n", errno, strerror(errno)); return 0; }
    printf("{\"io_uring_setup\": \"ok\", \"features\": %u, \"sq_entries\": %u}\n", p.features, p.sq_entries);
    close((int)fd);
    return 0;
}
