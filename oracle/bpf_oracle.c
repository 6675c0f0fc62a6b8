/*
 * bpf_oracle.c — CPU restatement of classic BPF evaluation as the reference's
 * pcap.BPF.Matches performs it.
 *
 * TEST INFRASTRUCTURE ONLY: loaded by tests/ and bench.py as the checker of
 * gopacket_amd/csrc/gpk_bpf.hip; nothing in gopacket_amd/ links or calls it.
 *
 * The reference (pcap/pcap.go:599-601 BPF.Matches -> pcap_unix.go:358-368
 * pcapOfflineFilter) hands the program to libpcap's pcap_offline_filter, i.e.
 * bpf_filter() over (packet, wirelen = ci.Length, buflen = len(data)).
 * libpcap is a third-party C dependency absent from /root/reference and from
 * this image (no pcap.h, no libpcap.so): this restates the published
 * algorithm of libpcap 1.10's bpf_filter.c (pcapint_filter_with_aux_data):
 *   - A, X and mem[16] start at 0; every packet load is big-endian and bounds
 *     checked against buflen, a failed check returns 0 (no match);
 *   - BPF_LEN loads wirelen; BPF_MSH loads 4 * (p[k] & 0xf);
 *   - DIV/MOD by X == 0 return 0; shifts by X >= 32 give 0;
 *   - JA adds the sign-extended k (ip6 protochain jumps backwards);
 *   - RET returns k or A; Matches = the return value != 0.
 * Where libpcap's C is undefined or aborts (unknown opcode: abort(); DIV/MOD
 * by a zero k; mem index >= 16; shift by a k >= 32; running past the last
 * instruction), this returns 0, except shifts by k, which use k & 31 (what the
 * x86 build does). Programs that never return are stopped after 1 << 20
 * instructions (0). Parity for those cases is unpinned by any reference vector.
 * Pinned: the reference's TestBPFInstruction programs and expected results on
 * pcap/test_ethernet.pcap (tests/golden/bpf_programs.json).
 */
#include <stdint.h>

#define BPF_CLASS(c) ((c) & 0x07)
#define BPF_LD 0x00
#define BPF_LDX 0x01
#define BPF_ST 0x02
#define BPF_STX 0x03
#define BPF_ALU 0x04
#define BPF_JMP 0x05
#define BPF_RET 0x06
#define BPF_MISC 0x07

typedef struct oracle_bpf_insn {
  uint16_t code;
  uint8_t jt, jf;
  uint32_t k;
} oracle_bpf_insn;

static uint32_t ld32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }
static uint32_t ld16(const uint8_t* p) { return (uint32_t)p[0] << 8 | p[1]; }

uint32_t oracle_bpf_filter(const oracle_bpf_insn* prog, uint32_t len, const uint8_t* p, uint32_t wirelen,
                           uint32_t buflen) {
  uint32_t A = 0, X = 0, k, mem[16] = {0};
  uint32_t pc = 0;
  for (uint32_t steps = 0; steps < (1u << 20); steps++) {
    if (pc >= len) return 0;
    const oracle_bpf_insn* i = &prog[pc];
    switch (i->code) {
      case 0x06: return i->k;                      /* RET K */
      case 0x16: return A;                         /* RET A */
      case 0x20:                                   /* LD W ABS */
        k = i->k;
        if (k > buflen || 4 > buflen - k) return 0;
        A = ld32(p + k);
        break;
      case 0x28:                                   /* LD H ABS */
        k = i->k;
        if (k > buflen || 2 > buflen - k) return 0;
        A = ld16(p + k);
        break;
      case 0x30:                                   /* LD B ABS */
        k = i->k;
        if (k >= buflen) return 0;
        A = p[k];
        break;
      case 0x80: A = wirelen; break;               /* LD W LEN */
      case 0x81: X = wirelen; break;               /* LDX W LEN */
      case 0x40:                                   /* LD W IND */
        k = X + i->k;
        if (i->k > buflen || X > buflen - i->k || 4 > buflen - k) return 0;
        A = ld32(p + k);
        break;
      case 0x48:                                   /* LD H IND */
        k = X + i->k;
        if (X > buflen || i->k > buflen - X || 2 > buflen - k) return 0;
        A = ld16(p + k);
        break;
      case 0x50:                                   /* LD B IND */
        k = X + i->k;
        if (i->k >= buflen || X >= buflen - i->k) return 0;
        A = p[k];
        break;
      case 0xb1:                                   /* LDX MSH B */
        k = i->k;
        if (k >= buflen) return 0;
        X = (uint32_t)(p[k] & 0xf) << 2;
        break;
      case 0x00: A = i->k; break;                  /* LD IMM */
      case 0x01: X = i->k; break;                  /* LDX IMM */
      case 0x60: if (i->k >= 16) return 0; A = mem[i->k]; break;  /* LD MEM */
      case 0x61: if (i->k >= 16) return 0; X = mem[i->k]; break;  /* LDX MEM */
      case 0x02: if (i->k >= 16) return 0; mem[i->k] = A; break;  /* ST */
      case 0x03: if (i->k >= 16) return 0; mem[i->k] = X; break;  /* STX */
      case 0x05: pc += i->k; break;                /* JA (k sign-extended: u32 wrap) */
      case 0x25: pc += (A > i->k) ? i->jt : i->jf; break;   /* JGT K */
      case 0x35: pc += (A >= i->k) ? i->jt : i->jf; break;  /* JGE K */
      case 0x15: pc += (A == i->k) ? i->jt : i->jf; break;  /* JEQ K */
      case 0x45: pc += (A & i->k) ? i->jt : i->jf; break;   /* JSET K */
      case 0x2d: pc += (A > X) ? i->jt : i->jf; break;      /* JGT X */
      case 0x3d: pc += (A >= X) ? i->jt : i->jf; break;     /* JGE X */
      case 0x1d: pc += (A == X) ? i->jt : i->jf; break;     /* JEQ X */
      case 0x4d: pc += (A & X) ? i->jt : i->jf; break;      /* JSET X */
      case 0x0c: A += X; break;                    /* ADD X */
      case 0x1c: A -= X; break;                    /* SUB X */
      case 0x2c: A *= X; break;                    /* MUL X */
      case 0x3c: if (X == 0) return 0; A /= X; break;  /* DIV X */
      case 0x9c: if (X == 0) return 0; A %= X; break;  /* MOD X */
      case 0x5c: A &= X; break;                    /* AND X */
      case 0x4c: A |= X; break;                    /* OR X */
      case 0xac: A ^= X; break;                    /* XOR X */
      case 0x6c: A = X < 32 ? A << X : 0; break;   /* LSH X */
      case 0x7c: A = X < 32 ? A >> X : 0; break;   /* RSH X */
      case 0x04: A += i->k; break;                 /* ADD K */
      case 0x14: A -= i->k; break;                 /* SUB K */
      case 0x24: A *= i->k; break;                 /* MUL K */
      case 0x34: if (i->k == 0) return 0; A /= i->k; break;  /* DIV K */
      case 0x94: if (i->k == 0) return 0; A %= i->k; break;  /* MOD K */
      case 0x54: A &= i->k; break;                 /* AND K */
      case 0x44: A |= i->k; break;                 /* OR K */
      case 0xa4: A ^= i->k; break;                 /* XOR K */
      case 0x64: A <<= (i->k & 31); break;         /* LSH K */
      case 0x74: A >>= (i->k & 31); break;         /* RSH K */
      case 0x84: A = 0u - A; break;                /* NEG */
      case 0x07: X = A; break;                     /* TAX */
      case 0x87: A = X; break;                     /* TXA */
      default: return 0;                           /* libpcap: abort() */
    }
    pc++;
  }
  return 0;
}

/* BPF.Matches over a packed batch: ret[i] = the filter's return value. */
void oracle_bpf_batch(const oracle_bpf_insn* prog, uint32_t len, const uint8_t* data, const uint64_t* offsets,
                      const uint32_t* caplens, const uint32_t* wirelens, uint64_t n, uint32_t* ret) {
  for (uint64_t i = 0; i < n; i++)
    ret[i] = oracle_bpf_filter(prog, len, data + offsets[i], wirelens ? wirelens[i] : caplens[i], caplens[i]);
}
