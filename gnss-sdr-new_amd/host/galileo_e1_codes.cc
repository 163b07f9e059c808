// Galileo E1-B / E1-C primary memory codes (Galileo OS SIS ICD Annex C) as a
// read-only table in the library: the bit-packed gsdr/data/galileo_e1_codes.bin
// (tools/extract_galileo_e1_codes.py; 100 rows -- E1-B PRN 1..50, then E1-C PRN
// 1..50 -- of 512 bytes, chip i at bit 7 - i%8 of byte i/8, logical 1 = chip -1),
// assembled in with .incbin (the Makefile puts the data directory on the
// assembler's include path).
asm(".pushsection .rodata\n"
    ".globl gsdr_galileo_e1_codes\n"
    ".type gsdr_galileo_e1_codes, @object\n"
    ".balign 16\n"
    "gsdr_galileo_e1_codes:\n"
    ".incbin \"galileo_e1_codes.bin\"\n"
    ".size gsdr_galileo_e1_codes, 51200\n"
    ".popsection\n");
