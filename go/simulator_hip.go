//go:build hip

// simulator_hip.go -- the cgo side of the MI355X engine, dropped next to the
// reference's simulator.go (package main).  It replaces the body of main()
// (simulator.go:207-253) once init() (:186-205) has parsed the flags; the
// seven flag globals N, Fanout, Fanin, DelayLow, DelayHigh, DropRate,
// CrashRate are the reference's own.
//
// Build (no Go toolchain ships in this repo's image; see INTEGRATION.md §2):
//
//	CGO_CFLAGS=-I<repo>/include \
//	CGO_LDFLAGS="-L<repo>/gossip_simulator_amd -lgossip_hip -Wl,-rpath,<repo>/gossip_simulator_amd" \
//	go build -tags hip
//
// and in simulator.go's main():  if useHIP { mainHIP(); return }
//
// Every C.gs_* name used here is declared in include/gossip.h; the CPU test
// tests/test_go_shim.py checks that (and the struct fields) on every run.
package main

/*
#include <stdlib.h>
#include "gossip.h"
*/
import "C"

import (
	"fmt"
	"runtime"
	"time"
	"unsafe"
)

func hipParams() C.gs_params {
	return C.gs_params{
		n: C.uint64_t(N), fanout: C.int32_t(Fanout), fanin: C.int32_t(Fanin),
		delay_low: C.int32_t(DelayLow), delay_high: C.int32_t(DelayHigh),
		drop_rate: C.double(DropRate), crash_rate: C.double(CrashRate),
		seed: 1, model: C.GS_MODEL_FLOOD, // C.GS_MODEL_PUSHPULL for the C5 extension
	}
}

func hipCheck(ctx *C.gs_ctx, rc C.int) {
	if rc == 0 {
		return
	}
	if ctx != nil {
		panic(C.GoString(C.gs_last_error(ctx)))
	}
	panic(C.GoString(C.gs_strerror(rc)))
}

func ms(t C.uint64_t) time.Duration { return time.Duration(t) * time.Millisecond }

// mainHIP replaces main() (simulator.go:207-253) on one GPU.
func mainHIP() {
	runtime.LockOSThread() // one gs_ctx is single-threaded
	p := hipParams()
	var ctx *C.gs_ctx
	hipCheck(nil, C.gs_create(&p, &ctx)) // :208-212
	defer C.gs_destroy(ctx)
	hipOverlay(ctx)
	hipBroadcast(ctx)
}

// hipOverlay replaces the stabilisation loop (simulator.go:214-235).
func hipOverlay(ctx *C.gs_ctx) {
	fmt.Println("\n=== Constructing Overlay ===") // :219
	win := make([]C.gs_window, 1<<16)
	var nwin C.size_t
	var stab C.uint64_t
	hipCheck(ctx, C.gs_build_overlay(ctx, 10000000, &win[0], C.size_t(len(win)), &nwin, &stab))
	if int(nwin) < len(win) {
		win = win[:int(nwin)]
	}
	for _, w := range win { // :230
		fmt.Println("break", w.breakups, "makeup", w.makeups, "elasped", ms(w.tick))
	}
	fmt.Printf("--- Took %v to stabilize ---\n\n", ms(stab)) // :235
}

// hipBroadcast replaces the broadcast and its poll loop (simulator.go:237-253).
func hipBroadcast(ctx *C.gs_ctx) {
	fmt.Println("=== Broadcast one message ===")  // :237
	hipCheck(ctx, C.gs_broadcast_begin(ctx, -1)) // :239-241
	var tot C.gs_tick_stats
	for { // :243-251
		hipCheck(ctx, C.gs_step(ctx, 10, nil))
		hipCheck(ctx, C.gs_totals(ctx, &tot))
		percent := float32(tot.received) / float32(N)
		fmt.Printf("%v%% covered, took %v\n", percent*100, ms(tot.tick))
		if percent >= 0.99 || tot.pending == 0 { // pending == 0: the reference would spin forever
			break
		}
	}
	fmt.Printf("--- Took %v to get 99%% ---\n\n", ms(tot.tick))
	fmt.Println("Total message", tot.messages, "Total Crashed", tot.crashed) // :253
}

// mainHIPSharded runs ONE broadcast with the node range split over several
// GPUs of this process (config C4); output is the same as mainHIP's.
func mainHIPSharded(devices []int32) {
	runtime.LockOSThread()
	p := hipParams()
	var ctx *C.gs_ctx
	hipCheck(nil, C.gs_create_multi(&p, (*C.int)(unsafe.Pointer(&devices[0])), C.int(len(devices)), &ctx))
	defer C.gs_destroy(ctx)
	hipOverlay(ctx)
	hipBroadcast(ctx)
}

// hipTrials runs `trials` independent broadcasts (config C3) batched on the
// given devices with no communication, and returns each trial's outcome --
// what one reference process prints at :252-253, once per trial.
func hipTrials(devices []int32, first, trials uint32) []C.gs_trial_stats {
	runtime.LockOSThread()
	p := hipParams()
	p.trial = C.uint32_t(first)
	p.trials = C.uint32_t(trials)
	var ctx *C.gs_ctx
	hipCheck(nil, C.gs_create_multi(&p, (*C.int)(unsafe.Pointer(&devices[0])), C.int(len(devices)), &ctx))
	defer C.gs_destroy(ctx)
	var nwin C.size_t
	var stab C.uint64_t
	hipCheck(ctx, C.gs_build_overlay(ctx, 10000000, nil, 0, &nwin, &stab))
	hipCheck(ctx, C.gs_broadcast_begin(ctx, -1))
	var status C.int32_t
	var nout C.size_t
	hipCheck(ctx, C.gs_run(ctx, 10, 10000000, nil, 0, &nout, &status))
	out := make([]C.gs_trial_stats, trials)
	hipCheck(ctx, C.gs_trial_results(ctx, &out[0], C.size_t(trials), &nout))
	return out[:int(nout)]
}

// hipCommID is called on rank 0 of a multi-process run; ship the bytes to
// every rank (any transport) before hipRank.
func hipCommID() []byte {
	id := make([]byte, C.GS_COMM_ID_BYTES)
	hipCheck(nil, C.gs_comm_unique_id((*C.uint8_t)(unsafe.Pointer(&id[0]))))
	return id
}

// hipRank is one process of a node-range-sharded run over nranks GPUs
// (config C4, RCCL all-gather per window inside libgossip_hip.so).  Every
// rank's gs_step/gs_totals return the global counters, so every rank may run
// the same poll loop; only rank 0 prints.
func hipRank(device, nranks, rank int, id []byte) {
	runtime.LockOSThread()
	p := hipParams()
	var ctx *C.gs_ctx
	hipCheck(nil, C.gs_create_rank(&p, C.int(device), C.int(nranks), C.int(rank),
		(*C.uint8_t)(unsafe.Pointer(&id[0])), &ctx))
	defer C.gs_destroy(ctx)
	var lo, hi C.uint64_t
	var nsh C.uint32_t
	hipCheck(ctx, C.gs_shard_info(ctx, 0, &nsh, &lo, &hi))
	var nwin C.size_t
	var stab C.uint64_t
	hipCheck(ctx, C.gs_build_overlay(ctx, 10000000, nil, 0, &nwin, &stab))
	hipCheck(ctx, C.gs_broadcast_begin(ctx, -1))
	var tot C.gs_tick_stats
	for {
		hipCheck(ctx, C.gs_step(ctx, 10, nil))
		hipCheck(ctx, C.gs_totals(ctx, &tot))
		percent := float32(tot.received) / float32(N)
		if rank == 0 {
			fmt.Printf("%v%% covered, took %v\n", percent*100, ms(tot.tick))
		}
		if percent >= 0.99 || tot.pending == 0 {
			break
		}
	}
	if rank == 0 {
		fmt.Printf("--- Took %v to get 99%% ---\n\n", ms(tot.tick))
		fmt.Println("Total message", tot.messages, "Total Crashed", tot.crashed)
	}
}
