/* rt_test_dll.c — console driver of the DLL API in plain C, linked against
 * libYulioRT_mi355x.so: the counterpart of the reference's rt_test_dll/rt_test_dll.cpp:12-44
 * (set ParamsRT, StartRT on a Collada file, WaitRT, report the status), with its optional
 * StopRT-after-N-seconds path (:36-39).
 *
 *   rt_test_dll <file.dae> [size] [spp] [--debug] [--watermark] [--stop-after <seconds>]
 *
 * Exit status 0 when the render finished (or was stopped on request) without an error. */
#define _POSIX_C_SOURCE 200809L
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "../../../include/YulioRT.h"

static const char* state_name(StateRT s) {
  switch (s) {
    case Inactive: return "Inactive";
    case Initialiazing: return "Initializing";
    case Rendering: return "Rendering";
    case Stopped: return "Stopped";
    case Done: return "Done";
  }
  return "?";
}

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s <file.dae> [size] [spp] [--debug] [--watermark] [--stop-after s]\n", argv[0]);
    return 2;
  }
  ParamsRT p;
  InitParamsRT(&p);
  double stopAfter = -1.0;
  int positional = 0;
  for (int i = 2; i < argc; ++i) {
    if (!strcmp(argv[i], "--debug")) p.debug = 1;
    else if (!strcmp(argv[i], "--watermark")) p.waterMark = 1;
    else if (!strcmp(argv[i], "--stop-after") && i + 1 < argc) stopAfter = atof(argv[++i]);
    else if (positional == 0) { p.size = atoi(argv[i]); positional++; }
    else if (positional == 1) { p.spp = atoi(argv[i]); positional++; }
  }
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  if (!StartRT(argv[1], &p)) {
    fprintf(stderr, "StartRT failed: error %d\n", (int)GetLastErrorRT());
    return 1;
  }
  int stopped = 0;
  if (stopAfter >= 0.0) {
    const struct timespec w = {(time_t)stopAfter, (long)((stopAfter - (double)(time_t)stopAfter) * 1e9)};
    nanosleep(&w, NULL);
    StatusRT s;
    GetCurrentStatusRT(&s);
    printf("after %.1f s: %s, progress %.3f\n", stopAfter, state_name(s.state), s.progress);
    stopped = StopRT(0) ? 1 : 0;
  } else {
    WaitRT();
  }
  clock_gettime(CLOCK_MONOTONIC, &t1);
  StatusRT s;
  GetCurrentStatusRT(&s);
  const double sec = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
  printf("state %s, progress %.3f, error %d, %.2f s (size %d, spp %d)\n", state_name(s.state), s.progress,
         (int)s.lastError, sec, p.size, p.spp);
  if (s.lastError != NoError) return 1;
  if (stopAfter >= 0.0) return (stopped && s.state == Stopped) ? 0 : 1;
  return s.state == Done ? 0 : 1;
}
