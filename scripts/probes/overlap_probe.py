"""Can a memory-bound adapter kernel overlap a hipBLASLt GEMM on a second stream?
Times GEMM alone, LoRA DOWN alone, and both issued on separate streams."""
import torch


def main():
    import lumen.ops.lora as L

    dev = torch.device("cuda")
    T, K, N = 4096, 4096, 12288
    x = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
    A = torch.randn(48, K, device=dev) * 0.01
    Z = torch.zeros(T, 48, device=dev)
    side = torch.cuda.Stream()

    def gemm():
        return x @ w.t()

    def down():
        Z.zero_()
        L._lora2(0, 1, x, A, Z, 48, 1, 1.0, T, 48, L._split(64, K, 256), [(0, 0, 0, K)], 7, 0.05, K)

    def timeit(fn, it=50):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(it):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / it * 1000

    def both():
        ev = torch.cuda.Event()
        ev.record()
        side.wait_event(ev)
        with torch.cuda.stream(side):
            for _ in range(4):
                down()
        y = gemm()
        torch.cuda.current_stream().wait_stream(side)
        return y

    def serial():
        for _ in range(4):
            down()
        return gemm()

    print(f"gemm {timeit(gemm):.1f} us, down {timeit(down):.1f} us, serial(gemm+4 down) "
          f"{timeit(serial):.1f} us, overlapped {timeit(both):.1f} us", flush=True)


if __name__ == "__main__":
    main()
