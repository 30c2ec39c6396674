# nanotel.R -- the R side of the MI355X hot path: wrappers over the .Call
# entry points of nanotel_r.c (libnanotel_r.so, linked against libnanotel.so)
# for NanoTel.R.  r/NanoTel.R.patch sources this file and replaces the
# per-chunk block of run_future_worker_chuncks (NanoTel.R:2234-2258: the 8
# forked search_patterns futures and their Reduce(union_all)) with
# nanotel_chunk(); everything else in NanoTel.R -- option parsing, the reader
# (readDNAStringSet, NanoTel.R:2213), reverseComplement (2219-2221), the
# summary.csv / reads_ids.txt writers and the log -- stays as it is.

nanotel_load <- function(lib = Sys.getenv("NANOTEL_R_LIB", "libnanotel_r.so")) {
  # one R process per GPU: HIP is initialised by nanotel_create() in this
  # process, so nothing may fork after it (future::multicore is not used)
  dyn.load(lib)
  invisible(TRUE)
}

# extract_patterns (NanoTel.R:2322-2334) and the fixed/IUPAC test (334) are
# the library's: the flags go in as given on the command line.  rc = FALSE
# when the caller reverse-complements the reads itself (as NanoTel.R does at
# 2219-2221, so that reads/*.fasta.gz hold the reads in scan orientation).
nanotel_create <- function(patterns, tvr_patterns = NULL, subseq_length = 100L,
                           min_density = 0.6, check_right_edge = FALSE, rc = FALSE,
                           device = 0L) {
  .Call("R_nt_create", as.integer(device), as.character(patterns),
        if (is.null(tvr_patterns)) NULL else as.character(tvr_patterns),
        as.integer(subseq_length), as.double(min_density),
        as.logical(check_right_edge), as.logical(rc))
}

nanotel_destroy <- function(nt) invisible(.Call("R_nt_destroy", nt))

# --use_filter: filter_reads + filter_density (NanoTel.R:2083-2163) for one
# chunk -- the reads it keeps, in order (NULL when none: the caller skips
# the chunk without touching serial_start, as NanoTel.R:2231 does)
nanotel_filter <- function(nt, dna_reads) {
  keep <- .Call("R_nt_filter_chunk", nt, as.character(dna_reads))
  if (!any(keep)) return(NULL)
  dna_reads[keep]
}

# One chunk: the rows analyze_read produces for every read of the chunk,
# serials and row order as the 8-way split and Reduce(union_all) give them
# (NanoTel.R:2050-2070, 2234-2254).  state: list(serial_start, max_serial),
# 1 and -Inf before the first chunk.  Returns list(rows, state, windows).
nanotel_analyze <- function(nt, dna_reads, state, want_windows = FALSE) {
  res <- .Call("R_nt_analyze_chunk", nt, as.character(dna_reads), names(dna_reads),
               as.double(state$serial_start), as.double(state$max_serial),
               as.logical(want_windows))
  list(rows = res$rows,
       state = list(serial_start = res$next_serial_start, max_serial = res$max_serial),
       windows = res$windows)
}

# The per-read files analyze_read writes for a row (NanoTel.R:1869-1918):
# reads/<serial>.fasta.gz and the three plots, drawn by NanoTel.R's own plot
# functions from the scan's window tables (analyze_list[[p]][[1]]) and the
# called positions (telo_position, telo_position2 [, telo_position3]).
nanotel_write_read <- function(row, win, dna_reads, output_dir, max_length = 1e5,
                               title = "Telomeric repeat density", tvr = FALSE) {
  serial <- row$Serial
  current_seq <- dna_reads[win$read]
  seq_len <- width(current_seq)
  output_jpegs <- paste(output_dir, "single_read_plots", sep = "/")
  output_jpegs_1 <- paste(output_dir, "single_read_plots_adj", sep = "/")
  fa <- paste(paste(output_dir, "reads", sep = "/"), paste(toString(serial), "fasta.gz", sep = "."), sep = "/")
  writeXStringSet(current_seq, fa, compress = TRUE)
  s <- win$start
  e <- win$end
  tb <- win$tables
  for (k in 1:3) {
    x_length <- if (k == 1) max_length else seq_len
    eps <- k == 3
    dir <- if (k == 1) output_jpegs else output_jpegs_1
    if (!tvr) {
      plot_single_telo_with_gray_area(x_length = x_length, seq_length = seq_len, subs = tb[[1]],
                                      subs_mismatch = tb[[2]], serial_num = serial,
                                      seq_start = s[1], seq_end = e[1], gray_start = s[2], gray_end = e[2],
                                      save_it = TRUE, main_title = title, w = 750, h = 300,
                                      output_jpegs = dir, eps = eps)
    } else {
      plot_single_telo_with_tvr(x_length = x_length, seq_length = seq_len, subs = tb[[1]],
                                subs_mismatch = tb[[2]], subs_tvr = tb[[3]], serial_num = serial,
                                seq_start = s[1], seq_end = e[1], gray_start = s[2], gray_end = e[2],
                                tvr_start = s[3], tvr_end = e[3], save_it = TRUE, main_title = title,
                                w = 750, h = 300, output_jpegs = dir, eps = eps)
    }
  }
}

# The replacement of NanoTel.R:2234-2258 for one chunk: rows appended to
# df_summary with union_all (as Reduce(union_all) does, 2254), the per-read
# files written, and the next chunk's serial state.
nanotel_chunk <- function(nt, dna_reads, df_summary, state, output_path, tvr_patterns = NULL) {
  res <- nanotel_analyze(nt, dna_reads, state, want_windows = TRUE)
  rows <- res$rows
  for (i in seq_len(nrow(rows))) {
    nanotel_write_read(rows[i, ], res$windows[[i]], dna_reads, output_path, tvr = !is.null(tvr_patterns))
  }
  list(df_summary = dplyr::union_all(df_summary, rows), state = res$state)
}
